# same-box comparison of the LM overlap modes (bench --overlap-mode), two runs each
mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT && \
for r in 1 2; do for m in 1 2 3 4; do
  timeout -k 10 300 python bench.py --cpu-baseline none --overlap-mode $m > gpurun_out/mode${m}_r$r.log 2>&1 || exit $?
done; done
