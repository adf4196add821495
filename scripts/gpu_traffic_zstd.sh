# config 5 memory-side traffic per kernel by request size (EA counters), one
# pass per counter group (scripts/traffic_summary.py, workload "c2" slot).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ztraffic}
mkdir -p $O
P1="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
P2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
P3="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/c2_p$i -- python bench.py --codec zstd --profile --steps 2 --warmup 1 > $O/c2_p$i.log 2>&1 || { tail -5 $O/c2_p$i.log; exit 1; }
done
python3 scripts/traffic_summary.py $O > $O/traffic.txt && cat $O/traffic.txt
