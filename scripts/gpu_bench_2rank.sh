# bench.py through torchrun with 2 ranks sharing the one GPU (collectives over gloo): exercises the
# multi-rank bench path (row chunks, async all-reduce, incremental sums per chunk) end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
CML_COMM_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/benches/bench_2rank_gloo.json 2> gpurun_out/benches/bench_2rank_gloo.err || { tail -30 gpurun_out/benches/bench_2rank_gloo.err; exit 1; }
cat gpurun_out/benches/bench_2rank_gloo.json | cut -c1-600
