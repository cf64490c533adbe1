# teardown probe matrix: (timing on/off) x (default wait / spin device flag)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02g
mkdir -p $OUT
timeout -k 10 120 python tools/probe_teardown.py > $OUT/td_default.json 2> $OUT/td.err || exit 1
timeout -k 10 120 python tools/probe_teardown.py --timing > $OUT/td_timing.json 2>> $OUT/td.err || exit 1
timeout -k 10 120 python tools/probe_teardown.py --spin > $OUT/td_spin.json 2>> $OUT/td.err || exit 1
timeout -k 10 120 python tools/probe_teardown.py --timing --spin > $OUT/td_timing_spin.json 2>> $OUT/td.err || exit 1
cat $OUT/td_*.json
