mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/b_async.log 2>&1 && \
YAVO_BUILD_PRIO=1 timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/b_prio.log 2>&1 && \
YAVO_BUILD_ASYNC=0 timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/b_sync.log 2>&1 && \
YAVO_BUILD_PRIO=1 timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/b_prio2.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/b_async2.log 2>&1
