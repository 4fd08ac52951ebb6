# same-box comparison of bench environment settings: each argument is one setting ("-" = defaults), two runs each
mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT || exit 1
for r in 1 2; do i=0; for e in "$@"; do i=$((i+1))
  if [ "$e" = "-" ]; then set_env=""; else set_env="$e"; fi
  env $set_env timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/env${i}_r$r.log 2>&1 || exit $?
done; done
