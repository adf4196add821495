# end-to-end zseek_pread (4 GiB into host memory, io 1 / 8) of two library
# builds, interleaved on one box: $1 output dir, $2 $3 libs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-e2eab}
mkdir -p $O
for r in 1 2; do
  for L in $2 $3; do
    ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/$L timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-latency --no-cpu-baseline > $O/e_$L_$r.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e_$L_$r.json')); print('$L', d['ms_per_step'], json.dumps(d['end_to_end']))"
  done
done
