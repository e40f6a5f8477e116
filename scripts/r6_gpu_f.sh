# probe experiments: the config-5 rank step with libcqgpu variants (PROBE_EXP)
set -e
OUT=gpurun_out/r6f; mkdir -p $OUT
for v in base p1 p2; do
  L=cq_amd/lib/libcqgpu.so; [ $v != base ] && L=cq_amd/lib/libcqgpu_$v.so
  CQ_AMD_LIB=$L CQ_AMD_TIMING=1 timeout -k 10 240 python scripts/r6_config5_profile.py --steps 3 > $OUT/$v.txt 2> $OUT/$v.err
  echo "$v $(python -c "import json;d=json.load(open('$OUT/$v.txt'));print(d['step_s']*1e3, d['phases_ms'], d['verified'])")"
  grep "typed kernels" $OUT/$v.err | tail -1
done
