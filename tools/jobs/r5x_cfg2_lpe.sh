# cfg2's one-launch rollout at 32 lanes per replica (2048 waves, default) vs 64 (4096 waves, MS_ENV_MIN_WAVES=4096)
O=gpurun_out/r5x; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline --steps 4 > $O/cfg2_lpe32_$i.json 2> $O/err.log || exit 1
  MS_ENV_MIN_WAVES=4096 timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline --steps 4 > $O/cfg2_lpe64_$i.json 2>> $O/err.log || exit 1
done
MS_ENV_MIN_WAVES=4096 timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fused_env_act" > $O/tests_lpe64.log 2>&1; echo "tests rc=$?" >> $O/job.log
