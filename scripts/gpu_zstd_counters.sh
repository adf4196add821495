# SQ counters of the one-frame zstd kernels over the latency probe (40
# requests): per-wave instructions and waits.  $1 output dir
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-zcnt}
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/p1 -- python scripts/latency_probe.py 40 zstd > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES --output-format csv -d $O/p2 -- python scripts/latency_probe.py 40 zstd > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
for k in zstd_seq_kernel zstd_huf_one zstd_frame_kernel seq_exec_frame; do python3 scripts/exec_counters.py $O $k mean; done
