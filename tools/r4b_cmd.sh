set -eo pipefail
bash tools/ab_variant.sh r4b own "env or kats or configs or compact or capture or many_groups"
O=gpurun_out/r4b
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --steps 2 > $O/cfg4_base$i.json 2> $O/cfg4_base$i.err
  MARLSCHED_LIB=$PWD/tools/_variants/own/libmarlsched.so timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --steps 2 > $O/cfg4_new$i.json 2> $O/cfg4_new$i.err
done
