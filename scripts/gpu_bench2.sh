set -o pipefail
# config 2 and config 5 bench lines (timed region uninstrumented)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/b2
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/b2/lz4.json 2> gpurun_out/b2/lz4.err || exit $?
timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/b2/zstd.json 2> gpurun_out/b2/zstd.err || exit $?
python - <<'P'
import json
for c in ("lz4", "zstd"):
    d = json.load(open(f"gpurun_out/b2/{c}.json")); r = d["roofline"]
    print(c, d["ms_per_step"], d["value"], r["frac"], {k: v["avg_ms"] for k, v in r["stages"].items()})
P
