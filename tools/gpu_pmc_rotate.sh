#!/bin/bash
# MFMA / LDS counters of the full-k restart rotation (k_rotate_stream, k = n_out = 128, N=1e8):
# two --pmc passes over the tuning tool's "rotate" op, each its own run.
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O/p1 $O/p2
cd /tmp && export TMPDIR=/tmp
T="$R/tools/tune_kernels.py run --variants ${VARIANTS:-base} --js 128 --ops rotate --rounds 1 --out $O/tune.json"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $T > $O/p1/out.txt 2>&1 || { echo "p1 failed"; tail $O/p1/out.txt; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_COEXEC_CYCLES FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $T > $O/p2/out.txt 2>&1 || { echo "p2 failed"; tail $O/p2/out.txt; exit 1; }
cd $R && python3 - $O <<'PY'
import csv, glob, sys, collections, json
O = sys.argv[1]
out = {}
for p in ("p1", "p2"):
    f = glob.glob(f"{O}/{p}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        if "k_rotate" not in r["Kernel_Name"]:
            continue
        acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"][:80]
    for d, c in acc.items():
        out.setdefault(names[d], []).append(dict(c))
summary = {}
for k, lst in out.items():
    keys = set().union(*lst)
    summary[k] = {n: sum(x.get(n, 0.0) for x in lst) / len(lst) for n in keys}
json.dump(summary, open(f"{O}/rotate_pmc.json", "w"), indent=1)
print(json.dumps(summary, indent=1))
PY
