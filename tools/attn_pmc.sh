cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && \
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY -d $R/gpurun_out/pmc1 --output-format csv -- python3 $R/tools/attn_bwd_bench.py 16384 2048 12 2 > $R/gpurun_out/p1.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmc2 --output-format csv -- python3 $R/tools/attn_bwd_bench.py 16384 2048 12 2 > $R/gpurun_out/p2.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmc3 --output-format csv -- python3 $R/tools/attn_bwd_bench.py 16384 2048 12 2 > $R/gpurun_out/p3.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -d $R/gpurun_out/pmc4 --output-format csv -- python3 $R/tools/attn_bwd_bench.py 16384 2048 12 2 > $R/gpurun_out/p4.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA -d $R/gpurun_out/pmc5 --output-format csv -- python3 $R/tools/attn_bwd_bench.py 16384 2048 12 2 > $R/gpurun_out/p5.log 2>&1 && \
cd $R && python3 tools/pmc_kernels.py gpurun_out/attn_pmc.json attn_fwd,attn_bwd_fused gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4 gpurun_out/pmc5
