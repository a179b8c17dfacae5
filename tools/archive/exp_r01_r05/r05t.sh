#!/bin/bash
# Round 5: the splice kernel's extension pops per lane per pass (HSA_SP_BUDGET 4 / 16 / 64) on config 4.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhsa_gpu.so libhsa_gpu_spb64.so libhsa_gpu_spb4.so libhsa_gpu.so; do
  n=${lib%.so}
  HSA_GPU_LIB=$lib timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --dropin 0 --ref-sample 0 \
      --parity-sample 1000 --cpu-sample 0 > gpurun_out/r05t_$n.json 2> gpurun_out/r05t_$n.err || { tail -5 gpurun_out/r05t_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05t_$n.json'));r=d['roofline'];print('$n', d['value'], r.get('k_search_ms'), r.get('splice_path_ms'), json.dumps(d.get('parity_sample'))[:100])"
done

HSA_GPU_LIB=libhsa_gpu_spdiag.so timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --dropin 0 --ref-sample 0 \
    --parity-sample 0 --cpu-sample 0 > gpurun_out/r05t_spdiag.out 2> gpurun_out/r05t_spdiag.err || { tail -5 gpurun_out/r05t_spdiag.err; exit 2; }
grep "sp_diag" gpurun_out/r05t_spdiag.out | tail -3 | cut -c1-300
echo diag done
