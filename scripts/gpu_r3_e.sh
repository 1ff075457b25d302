# Round 3 batch e: where the halo pack's time goes -- pack-only, unpack-only and pair loops,
# with and without a cold-clean flush, for the halo (cfg2) and its two x faces (xx), 16 fields
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r3e_halo_split.jsonl
for c in cfg2 xx; do
  for m in pair pack unpack; do
    for fl in none read; do
      timeout -k 10 200 python3 scripts/ab.py --config $c --rounds 3 --steps 20 --mode $m --flush $fl --variants "snt=-1" >> gpurun_out/r3e_halo_split.jsonl 2>gpurun_out/r3e.err || exit $?
    done
  done
done
timeout -k 10 300 python3 scripts/ab.py --config cfg2 --rounds 3 --steps 20 --mode pair --variants "wt=-1,wt=0,wt=2,nt=0,nt=1,xcd=0,xcd=1" >> gpurun_out/r3e_halo_variants.jsonl 2>>gpurun_out/r3e.err
cut -c1-200 gpurun_out/r3e_halo_split.jsonl gpurun_out/r3e_halo_variants.jsonl
