#!/bin/bash
# Round 6: the NTT engine's radix plan (radix 32 on the unit pass): parity
# of every NTT-engine path, then A/B bench lines against the round-5 plan
# (build/ab/ntt_r5, tools/ab/ntt_plan_r5.patch).
set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_fec_vector.py tests/test_kernel_names.py -m gpu -v --timeout 300 --timeout-method thread -k "batch_vs_oracle or golden or general_path or eras or ntt or unaligned or lazy or bad_ids or dense or overflow or streams or fec_vector or kernels_exist" > $O/pytest_ntt.log 2>&1 || { tail -30 $O/pytest_ntt.log; exit 1; }
tail -1 $O/pytest_ntt.log
AB_WARMUP=30 bash tools/ab_quick.sh r6i "k600 k1000" ntt_r5
