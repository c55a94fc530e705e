set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
run() { echo "== $*"; timeout -k 10 120 "$@" || exit 1; }
run python -u benchmarks/head_bench.py --iters 30
FEDREC_HEAD_WG=1 run python -u benchmarks/head_bench.py --iters 30
FEDREC_HEAD_SPLITS=14 run python -u benchmarks/head_bench.py --iters 30
FEDREC_HEAD_SPLITS=56 run python -u benchmarks/head_bench.py --iters 30
O=$PWD/gpurun_out/pmc_head; rm -rf $O; mkdir -p $O
timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d $O -o p1 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- python benchmarks/head_bench.py --iters 5 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d $O -o p2 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -- python benchmarks/head_bench.py --iters 5 > $O/p2.log 2>&1 || exit 1
python - <<'PY'
import csv, collections, glob
for p in ("p1","p2"):
    f=glob.glob(f"gpurun_out/pmc_head/{p}_counter_collection.csv")
    if not f: print("no", p); continue
    agg=collections.defaultdict(lambda: collections.defaultdict(float)); dur=collections.defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        n=r["Kernel_Name"][:60]
        agg[n][r["Counter_Name"]]+=float(r["Counter_Value"])
        dur[n][r["Dispatch_Id"]]=int(r["End_Timestamp"])-int(r["Start_Timestamp"])
    for n,c in agg.items():
        print(p, n, "disp", len(dur[n]), "ns", sum(dur[n].values())//max(1,len(dur[n])), {k: round(v/len(dur[n])) for k,v in c.items()})
PY
