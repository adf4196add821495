# round 4 evidence, second half (config 5, config 3 sweep, compression lines,
# PCIe probe) after the first run stopped at the config-5 trace (tools
# libzstd fix, see tools.cpp).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/round4
Z=gpurun_out/zround4
S=gpurun_out/sweep4
mkdir -p $O $Z $S
timeout -k 10 600 python bench.py --codec zstd > $Z/bench.json 2> $Z/bench.err && cat $Z/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $Z/trace -- python bench.py --codec zstd --profile --steps 5 --warmup 1 > $Z/trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $Z/pmc_fetch -- python bench.py --codec zstd --profile --steps 2 --warmup 1 > $Z/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $Z/pmc_write -- python bench.py --codec zstd --profile --steps 2 --warmup 1 > $Z/pmc_write.log 2>&1 &&
echo "config 5 profiles done" &&
timeout -k 10 400 python bench.py --frame 4096 --steps 5 --warmup 2 --no-e2e > $S/f4096.json 2> $S/f4096.err && cat $S/f4096.json &&
timeout -k 10 400 python bench.py --frame 1048576 --steps 5 --warmup 2 --no-e2e > $S/f1048576.json 2> $S/f1048576.err && cat $S/f1048576.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $S/trace1m -- python bench.py --frame 1048576 --profile --steps 5 --warmup 1 > $S/trace1m.log 2>&1 &&
timeout -k 10 400 python bench.py --codec lz4c --steps 3 --warmup 1 > $S/lz4c.json 2> $S/lz4c.err && cat $S/lz4c.json &&
timeout -k 10 400 python bench.py --codec lz4c --frame 1048576 --size 1073741824 --steps 3 --warmup 1 > $S/lz4c_1m.json 2> $S/lz4c_1m.err && cat $S/lz4c_1m.json &&
timeout -k 10 200 python scripts/pcie_probe.py > $O/pcie.json 2> $O/pcie.err && cat $O/pcie.json
rc=$?
exit $rc
