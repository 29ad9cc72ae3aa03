#!/bin/bash
# Round-3 batch 1: paired-M0 DMA issue (impl 22), v8 intra-CU stagger, resident-CU reserve,
# the forced N > 1 paths.
steps=("300:r3_gputest_new:python -u -m pytest tests/test_gemm_table_gpu.py -q -k 'cu_reserve or paired' --timeout 120 --timeout-method thread"
       "300:ab22_gpt2s:python -u bench/gemm_ab.py --shapes gpt2s --impls 20 22 23 21 --rounds 3 --iters 5"
       "300:ab22_sq:python -u bench/gemm_ab.py --shapes square --impls 20 22 23 --rounds 3 --iters 3"
       "200:cu_reserve:python -u bench/cu_reserve.py")
for ns in 0 4000; do
  steps+=("200:st8_fused_$ns:env DPC_G8_STAGGER_NS=$ns python -u bench/gemm_ab.py --shapes fused --impls 20 21 --rounds 3 --iters 5")
done
steps+=("150:fd_ddp_base:python -u bench.py"
        "150:fd_ddp:python -u bench.py --force_dist_path"
        "150:fd_ddp_eager:python -u bench.py --force_dist_path --no_graph"
        "200:fd_fsdp_base:python -u bench.py --recipe fsdp --steps 8 --warmup 3"
        "200:fd_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3 --force_dist_path"
        "200:fd_ppd_base:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3"
        "200:fd_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3 --force_dist_path")
scripts/gpu_step.sh "${steps[@]}"
