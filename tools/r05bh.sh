export TMPDIR=/tmp; O=gpurun_out/r05bh
TAG=r05bh bash tools/gpu_task.sh benchpmc || exit 1
python - <<'PY' || exit 1
import json
for n in ("pmc_traffic", "pmc_valu"):
    new = json.load(open(f"gpurun_out/r05bh/{n}.json")); cur = json.load(open(f"profiles/{n}.json"))
    cur.update(new); json.dump(cur, open(f"profiles/{n}.json", "w"), indent=1)
    cur.update(new); json.dump(cur, open(f"gpurun_out/r05bh/{n}_merged.json", "w"), indent=1)
PY
TAG=r05bh bash tools/gpu_task.sh trace smoke bench
