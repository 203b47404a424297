# Round 5: the 3D GPU tests with the staging rings (StageRing) library.
set -u
O=gpurun_out/r5ae
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_fast3d_gpu.py \
  tests/test_threading_gpu.py tests/test_constraint_builder_3d.py tests/test_ties_walk.py tests/test_ceres3d.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
