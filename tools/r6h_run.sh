set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "cfg2_full_batch or dense_tiles_spread or bucket_overflow" > $O/pytest_new.log 2>&1 || { tail -30 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
QI_LIB_PATH=build/ab/ctx512/libquadiron_amd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "cfg3 or batch_vs_oracle or golden or row_scales or dense" > $O/pytest_ctx512.log 2>&1 || { tail -30 $O/pytest_ctx512.log; exit 1; }
tail -1 $O/pytest_ctx512.log
for v in main ctx512; do L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
  QI_LIB_PATH=$L timeout -k 10 120 python3 tools/ctx_time.py 64,960,1024,2048 48,976,1024,2048 > $O/ctx_$v.txt 2>&1 || exit 1; echo $v; cat $O/ctx_$v.txt; done
AB_WARMUP=60 bash tools/ab_quick.sh r6h "cfg3" ctx512
