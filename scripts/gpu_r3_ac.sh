# Round 3 batch ac: 8-byte gather cost by load coherence scope (scripts/ubench_ldpol.hip), timing
# and the L2's read-request sizes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench_ldpol 10 > gpurun_out/r3ac_ubench_ldpol.log 2>&1 || exit $?
cat gpurun_out/r3ac_ubench_ldpol.log
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/r3ac_pmc -o pmc -- ./scripts/ubench_ldpol 2 > gpurun_out/r3ac_pmc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r3ac_pmc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "gather" in k:
        acc[(k[:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:40s} {c:24s} per launch {sum(v)/len(v)/ (2<<20):.3f} per line ({len(v)} launches)")
PY
