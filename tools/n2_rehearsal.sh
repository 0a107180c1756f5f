cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --steady-batches 1 > gpurun_out/n2.log 2>&1; echo rc=$?
tail -c 1500 gpurun_out/n2.log
