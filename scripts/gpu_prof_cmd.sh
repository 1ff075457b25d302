# e2e host-resident rates + rocprofv3 evidence for the bench line
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/e2e.log
for c in cfg2 cfg1 cfg3; do
  timeout -k 10 300 python scripts/e2e.py --config $c >> gpurun_out/e2e.log 2>&1 || exit $?
done
grep -h config gpurun_out/e2e.log | cut -c1-600
CFG=cfg2 timeout -k 10 1000 bash scripts/profile_round.sh
