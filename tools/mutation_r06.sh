# Mutation builds of the three-slot short-batch pipeline (gx_api_batch.cpp trace_dev):
#   mut_nowait: no hipStreamWaitEvent(tstream, fdone) before the walk on its own stream
#   mut_early:  the fill's buffers go back to the pool as soon as the walk is queued
# Each must fail tests/test_gpu_atsize.py::test_short_pipeline_alternating_sets (exit 1 = tests failed).
mkdir -p gpurun_out
for M in mut_nowait mut_early; do
  GX_LIB=genomics-rs_amd/build_var/libgx_amd_$M.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_atsize.py -k short_pipeline -m gpu > gpurun_out/r06_$M.log 2>&1
  rc=$?
  echo "$M exit $rc" >> gpurun_out/r06_mutations.txt
  [ $rc -le 1 ] || exit $rc   # (anything but pass / test failure: stop)
done
