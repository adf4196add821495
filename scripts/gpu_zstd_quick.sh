set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05zq
mkdir -p $O
timeout -k 10 120 rocprofv3 --list-avail > $O/avail.txt 2>&1; grep -i -E "dram|mall|TCC_EA0_RD|HBM" $O/avail.txt | head -40
timeout -k 10 300 python bench.py --codec zstd --steps 5 --warmup 2 --no-e2e --no-latency --no-cpu-baseline > $O/bench.json 2> $O/bench.err && python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step']); print(json.dumps(d['roofline']['stages'], indent=0)); print(d['roofline']['dominant_kernel'])"
