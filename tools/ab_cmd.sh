# same-box A/B of one bench knob: default vs the environment assignment given as $1 (e.g. YAVO_BUILD_ASYNC=0)
mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 python bench.py > gpurun_out/ab_a1.log 2>&1 && \
env $1 timeout -k 10 300 python bench.py > gpurun_out/ab_b1.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/ab_a2.log 2>&1 && \
env $1 timeout -k 10 300 python bench.py > gpurun_out/ab_b2.log 2>&1
