# GPU suite + two default bench runs (stops at the first failure)
mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/q_b1.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/q_b2.log 2>&1
