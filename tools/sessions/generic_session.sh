set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_module.py tests/test_descriptor.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -4 || exit 1
for p in 3 0; do
  DSPB_STATELESS_PATH=$p timeout -k 10 200 python -u tools/generic_probe.py 10 gain_test IR_test handmade_test no_op || exit 1
  DSPB_STATELESS_PATH=$p timeout -k 10 200 python -u tools/generic_probe.py 3600 gain_test IR_test handmade_test no_op || exit 1
done
