# Lean parse bring-up: GPU parity suite, then kbench A/B on config 2
# (79 default = lz4_lean_kernel + execute v13, 89 = older scan parse,
# 83 plan + lean parse, 87/88 lean diagnostics: no line stores / one line).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lean_pytest.log 2>&1 &&
tail -3 gpurun_out/lean_pytest.log &&
timeout -k 10 300 python -u scripts/kbench.py --variants ${VARIANTS:-79,89,83,87,88} --rounds 3 --reps 3 > gpurun_out/lean_kbench.log 2>&1
rc=$?
tail -3 gpurun_out/lean_pytest.log
cat gpurun_out/lean_kbench.log
exit $rc
