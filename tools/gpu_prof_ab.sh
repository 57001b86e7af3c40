# rocprofv3 kernel stats of the headline step under two env settings: bash tools/gpu_prof_ab.sh "A=0" "A=1"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for envs in "$@"; do
  rm -rf gpurun_out/profab$i
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profab$i -o run -- python bench.py --steps 5 --warmup 3 > gpurun_out/profab$i.log 2>&1 || { tail -20 gpurun_out/profab$i.log; exit 1; }
  f=$(find gpurun_out/profab$i -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kernel_stats_ab$i.csv
  rm -rf gpurun_out/profab$i
  i=$((i+1))
done
python - "$@" <<'PY'
import csv, sys
envs = sys.argv[1:]
tabs = []
for i in range(len(envs)):
    rows = list(csv.DictReader(open(f"gpurun_out/kernel_stats_ab{i}.csv")))
    tabs.append({r["Name"][:70]: float(r["TotalDurationNs"]) / 8e6 for r in rows})
names = sorted(set().union(*tabs), key=lambda n: -tabs[0].get(n, 0))
print("ms/step".rjust(8), " | ".join(e.rjust(14) for e in envs))
for n in names[:18]:
    print(n.ljust(70), " | ".join(f"{t.get(n, 0):14.3f}" for t in tabs))
print("TOTAL".ljust(70), " | ".join(f"{sum(t.values()):14.3f}" for t in tabs))
PY
