#!/bin/bash
# round 3e: GMRES host-poll A/B, device-resident time loop (tests + A/B), driver and GMRES tests
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 python tools/ab_gmres.py --no-prof --rounds 5 --variants gm_poll_every=1,gm_poll_every=2,gm_poll_every=4,gm_poll_every=30 > gpurun_out/ab_gm_poll.txt 2>&1 || exit $?
echo "poll A/B done"
timeout -k 10 600 $T tests/test_cpp_driver.py tests/test_reference_inputs.py -m gpu > gpurun_out/r03e_driver_tests.log 2>&1 || { tail -30 gpurun_out/r03e_driver_tests.log; exit 1; }
echo "driver tests done"
timeout -k 10 400 $T tests/test_gpu_gmres.py tests/test_gpu_fa.py -k gmres > gpurun_out/gm_tests.log 2>&1 || { tail -30 gpurun_out/gm_tests.log; exit 1; }
echo "gmres tests done"
timeout -k 10 600 bash tools/ab_time_loop.sh 256 3 > gpurun_out/ab_time_loop.txt 2>&1 || { tail -5 gpurun_out/ab_time_loop.txt; exit 1; }
echo "time loop A/B done"
