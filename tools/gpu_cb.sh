# N > 1 rehearsal after this session's routing changes: gloo, 2 ranks on the one GPU
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ENSVS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 > gpurun_out/cb_gloo2.json 2> gpurun_out/cb_gloo2.err || exit 1
