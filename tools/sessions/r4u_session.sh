# Round 4: 2-rank rehearsal of the multi-GPU bench path on one GPU (gloo,
# TCP communicator) at HEAD, then the 2/3-rank RCCL stand-in tests.
set -u
O=gpurun_out/r4u
mkdir -p $O
bash tools/gpu_measure.sh $O gloo2 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('$O/rehearsal_2rank.json') if l.startswith('{')][-1])
print({k: d[k] for k in ('value','n_gpus','ms_per_step','accepted_constraints','errors_per_step','chunks_claimed','chunks_max_rank') if k in d})"
timeout -k 10 400 python -u -m pytest tests/test_comm_rccl_gpu.py tests/test_distributed.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_dist.log 2>&1 || { tail -40 $O/tests_dist.log; exit 1; }
tail -1 $O/tests_dist.log
