# one-GPU rehearsal of bench.py's N > 1 control flow (gloo, every rank on cuda:0) + GEMM A/B
bash tools/gpu_session.sh \
 "rehearse2:420:PRL_BENCH_REHEARSE=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --tokens 16384 --no-trainer-step" \
 "gemm_base:200:python tools/gemm_shapes_bench.py 65536 1.5b" \
 "gemm_tuned:200:PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=tools/tunableop.csv python tools/gemm_shapes_bench.py 65536 1.5b"
