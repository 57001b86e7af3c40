set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/blt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/blt -o run -- python tools/blt_probe.py > gpurun_out/blt.log 2>&1 || { tail -20 gpurun_out/blt.log; exit 1; }
find gpurun_out/blt -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -c1-400 {}
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
