#!/bin/bash
# Round-5 GPU step: the named test files, then optional A/B / bench commands, each under its own limit.
# usage: TAG=x TESTS="tests/a.py tests/b.py" AB="--n 128 --p 4 --iters 20 --variant ho_brick=0 --variant ho_brick=1" \
#        BENCH="--config c3 --steps 3" bash tools/gpu_r05.sh
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r05}; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q --maxfail 10 --timeout 300 --timeout-method thread -p no:cacheprovider \
      > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed|Error" $O/tests.log | head -30; exit 1; }
  tail -2 $O/tests.log
fi
if [ -n "${AB:-}" ]; then
  timeout -k 10 900 python -u tools/ab_opts.py $AB > $O/ab.json 2> $O/ab.err || { echo "ab rc=$?"; tail $O/ab.err; exit 1; }
  cat $O/ab.json
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('%.4e'%d['value'], d['ms_per_step'], r['bound'], r['frac'], r['avg_launch_us'], r['other_kernels_avg_us'])"
fi
if [ -n "${MRLIST:-}" ]; then  # kernel launches per iteration: one rank, 2 ranks folded / not folded
  for cfg in "1 1" "2 1" "2 0" "3 1"; do set -- $cfg
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/mr_w$1_f$2 -o run --output-format csv -- python3 tools/mr_kernel_list.py --world $1 --fold $2 > $O/mr_w$1_f$2.log 2>&1 || { echo "mr $cfg rc=$?"; tail $O/mr_w$1_f$2.log; exit 1; }
    python3 tools/mr_kernel_list.py --summary $O/mr_w$1_f$2 --world $1 --fold $2 | tee -a $O/mr_kernel_list.jsonl
  done
fi
exit 0
