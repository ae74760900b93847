# One-GPU rehearsal of bench.py's N > 1 control flow: every rank on cuda:0 over gloo
# (PRL_BENCH_REHEARSE=gloo; small split / FSDP shapes).  Timings are meaningless; it checks that
# every probe of the N = 2, 4 and 8 bench lines completes and verifies its result (the N > 1 line's
# "communicators" census reports gloo sizes there; the prl_comm communicator needs one GPU per rank).
bash tools/gpu_session.sh \
 "rehearse2:600:PRL_BENCH_REHEARSE=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --tokens 16384" \
 "rehearse4:900:PRL_BENCH_REHEARSE=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 5 --warmup 2 --tokens 16384" \
 "rehearse8:1100:PRL_BENCH_REHEARSE=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 5 --warmup 2 --tokens 16384"
