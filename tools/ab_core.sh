for v in libfdr libfdr_nt libfdr_u8 libfdr_ntu8; do
  for c in impala impala_fp16; do
    FDR_LIB=$PWD/dfd-starter_amd/fdr/$v.so timeout -k 10 200 python bench.py --config $c --episode-len 100 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { echo "$v $c FAIL"; tail -3 gpurun_out/ab.log; continue; }
    tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v $c conv %.3f core %.3f frac %.3f' % (r['conv_launch_ms'], r['core_kernel']['launch_ms'], r['core_kernel']['frac']))"
  done
done
