# GEMM epilogue change check: kernel tests (bf16 + fp8 epilogues), LDS bank-conflict counters of the NT kernel, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp G1_T=131072
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_fp8.py tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/epi_tests.log 2>&1 || { tail -30 gpurun_out/epi_tests.log; exit 1; }
tail -2 gpurun_out/epi_tests.log
rm -rf gpurun_out/pmc_epi
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_epi -o run -- python tools/gemm2_one.py fwd > gpurun_out/pmc_epi.log 2>&1 || { tail -10 gpurun_out/pmc_epi.log; exit 1; }
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_epi/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm2" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: f"{sum(v)/len(v):.4g}" for k, v in agg.items()})
PY
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
