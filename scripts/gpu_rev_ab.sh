# reverse task order A/B (ddt_tune rev) in the pack+unpack pair loop.
# Historical: the knob was removed after this A/B showed no gain (profiles/r1_rev_ab.log).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/rev_ab.log
for c in cfg2 xx yz cfg3 cfg5 cfg1; do
  timeout -k 10 300 python scripts/ab.py --config $c --mode pair --variants "rev=0,rev=1,rev=2" --rounds 3 >> gpurun_out/rev_ab.log 2>&1 || exit $?
done
grep -h variant gpurun_out/rev_ab.log | cut -c1-120
