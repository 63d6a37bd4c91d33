# cfg4's env round at 16 lanes per replica (2048 waves, default) vs 32 (4096 waves, MS_ENV_MIN_WAVES=4096, generic shape)
O=gpurun_out/r6v; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/lpe16_$i.json 2>> $O/err.log || exit 1
  MS_ENV_MIN_WAVES=4096 timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/lpe32_$i.json 2>> $O/err.log || exit 1
done
