set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do timeout -k 10 300 python -X faulthandler -m pytest tests/test_gpu_zstd.py -x -q -m gpu > gpurun_out/pt_zstd$i.log 2>&1 || { grep -v "^Extension" gpurun_out/pt_zstd$i.log | tail -20; exit 1; }; tail -1 gpurun_out/pt_zstd$i.log; done
ZSEEK_ZSTD_TIMING=1 timeout -k 10 600 python bench.py --codec zstd --no-e2e --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bench_zstd.json 2> gpurun_out/bench_zstd.err; rc=$?; python -c "import json; d=json.load(open('gpurun_out/bench_zstd.json')); print(d['value'], d['roofline']['stages'])"; grep "zstd frame kernel" gpurun_out/bench_zstd.err | tail -1; exit $rc
