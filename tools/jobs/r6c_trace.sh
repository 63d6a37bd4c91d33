# kernel trace of graph-replayed cfg3 iterations (per-iteration census of the update's small kernels)
O=$PWD/gpurun_out/r6c; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-step-kernel --no-cpu-baseline > $O/bench.json 2> $O/bench.err
