# GPU LZ4 compression: parity tests + one bench line (A/B iterations)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lz4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lz4_compress.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --codec lz4c --steps 5 --warmup 2 --no-cpu-baseline > $O/quick.json 2> $O/quick.log || { tail -20 $O/quick.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/quick.json'));print(d['value'],d['ms_per_step'],d['verified_bit_exact'])"
