set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "golden_tables or fp32_bit_exact or known_answer or repeated or max_sweeps or invalid" > gpurun_out/pytest_vi1.log 2>&1
echo "exit $?"
