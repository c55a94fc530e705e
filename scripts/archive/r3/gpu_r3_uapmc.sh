set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT:$PYTHONPATH
O=$PWD/gpurun_out/pmc_ua; rm -rf $O; mkdir -p $O
timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d $O -o p1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -- python benchmarks/user_attn_bench.py --rounds 1 > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
python - <<'PY'
import csv, collections, glob
f=glob.glob("gpurun_out/pmc_ua/p1_counter_collection.csv")[0]
agg=collections.defaultdict(lambda: collections.defaultdict(float)); dur=collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    n=r["Kernel_Name"][:50]
    agg[n][r["Counter_Name"]]+=float(r["Counter_Value"])
    dur[n][r["Dispatch_Id"]]=int(r["End_Timestamp"])-int(r["Start_Timestamp"])
for n,c in agg.items():
    if "user_attn" not in n: continue
    d=len(dur[n]); print(n, "disp", d, "ns", sum(dur[n].values())//d, {k: round(v/d) for k,v in c.items()})
PY
