# cfg4: each unit type's update on its own stream (MS_UPDATE_STREAMS=1) vs one stream
O=gpurun_out/r6o; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/one_$i.json 2>> $O/err.log || exit 1
  MS_UPDATE_STREAMS=1 timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/streams_$i.json 2>> $O/err.log || exit 1
done
