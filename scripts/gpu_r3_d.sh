# Round 3 batch d: streaming-leaf policy A/B under the cold-clean (read-flush) face protocol
set -o pipefail
mkdir -p gpurun_out
V="snt=-1,snt=3,snt=1,snt=5,stask=8192,snt=3;stask=8192,snt=5;stask=8192"
for f in y z; do
  for fl in read none; do
    timeout -k 10 300 python3 scripts/ab.py --config $f --count 512 --rounds 3 --steps 10 --flush $fl --variants "$V" >> gpurun_out/r3d_ab.jsonl 2>gpurun_out/r3d_ab.err || exit $?
  done
done
cut -c1-220 gpurun_out/r3d_ab.jsonl
