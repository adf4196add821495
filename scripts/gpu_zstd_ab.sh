# config 5 A/B of two builds of the library (ZSEEK_AMD_LIB), interleaved,
# plus the zstd GPU tests on the production build: $1 output dir, $2 $3 libs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-zab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_zstd.py > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for r in 1 2; do
  for L in $2 $3; do
    ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/$L timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-latency --no-cpu-baseline > $O/b_$L_$r.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/b_$L_$r.json')); print('$L', d['ms_per_step'], json.dumps({k: v.get('median_ms') for k, v in (d['roofline'].get('stages') or {}).items()}))"
    ZSEEK_ZSTD_SERIAL=1 ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/$L timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-latency --no-cpu-baseline > $O/s_$L_$r.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/s_$L_$r.json')); print('$L serial', d['ms_per_step'], json.dumps({k: v.get('median_ms') for k, v in (d['roofline'].get('stages') or {}).items()}))"
  done
done
