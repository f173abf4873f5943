set -u
# gm_vec2 (16-byte basis pairs in the CGS passes): GMRES parity, then the in-process GMRES A/B at C2
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_gmres.py --durations=5 > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_gmres.py --rounds 4 --iters 60 --variants "gm_vec2=0,gm_vec2=1" > $O/ab_ev.json 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_gmres.py --rounds 4 --iters 60 --no-prof --variants "gm_vec2=0,gm_vec2=1" > $O/ab_noev.json 2>&1 || exit $?
