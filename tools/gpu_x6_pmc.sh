# PMC counters of the split-bf16 GEMM on a 512-tile shape (no wave quantisation) vs x3 / native / library
cd /tmp && export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/x6pmc
for e in x6 x3 native blas; do
timeout -k 10 120 python3 $R/tools/bench_gemm_x6.py --only 4096,2048,768,0,1,$e --reps 50 || exit 1
timeout -k 10 120 python3 $R/tools/bench_gemm_x6.py --only 4096,2048,3072,0,0,$e --reps 50 || exit 1
done
for e in x6 x3; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/x6pmc/a_$e -o run -- python3 $R/tools/bench_gemm_x6.py --only 4096,2048,768,0,1,$e --reps 10 > $R/gpurun_out/x6pmc/a_$e.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/x6pmc/b_$e -o run -- python3 $R/tools/bench_gemm_x6.py --only 4096,2048,768,0,1,$e --reps 10 > $R/gpurun_out/x6pmc/b_$e.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, os, collections
R = os.environ["GRAFT_REPO_ROOT"]
for f in sorted(glob.glob(R + "/gpurun_out/x6pmc/*/run_counter_collection.csv")):
    agg = collections.defaultdict(float); ns = {}; gui = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "gemm_x6s" not in r["Kernel_Name"]: continue
        d = r["Dispatch_Id"]; ns[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE": gui[d] = max(gui[d], float(r["Counter_Value"]))
        else: agg[r["Counter_Name"]] += float(r["Counter_Value"])
    n = len(ns); t = sum(ns.values()) / n
    print(f.split("/")[-2], "dispatches", n, "avg us %.1f" % (t / 1e3), "clock GHz %.2f" % (sum(gui.values()) / n / t),
          " ".join("%s=%.4g" % (k, v / n) for k, v in sorted(agg.items())))
PY
