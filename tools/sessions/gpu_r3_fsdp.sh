#!/bin/bash
# fused FSDP step collective + calibration + GELU/LN changes: targeted tests, then benches
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/fsdp
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_kernels_gpu.py -k "fsdp_over_xgmi or xgmi_collectives or ln_gemm or attn128 or gemm" -x -q --timeout 200 --timeout-method thread > gpurun_out/fsdp/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/fsdp/pytest.log; [ $rc -ne 0 ] && exit $rc
for a in "--strategy pp --model transformer" "--strategy pp --model transformer --microbatch-passes"; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 $a > gpurun_out/fsdp/b.log 2>&1 || { tail -3 gpurun_out/fsdp/b.log; exit 1; }
  echo "'$a': $(grep '^{' gpurun_out/fsdp/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
export JDT_BACKEND=gloo
for a in "--strategy fsdp" "" "--strategy fsdp --num-layers 4"; do
  for f in 1 0; do
    [ "$a" = "" ] && [ $f -eq 0 ] && continue
    JDT_FSDP_FUSED_COMM=$f timeout -k 10 240 python bench.py --gpus 2 --steps 200 --warmup 20 $a > gpurun_out/fsdp/b2.log 2>&1 || { tail -5 gpurun_out/fsdp/b2.log; exit 1; }
    echo "N=2 '$a' fused_comm=$f: $(grep '^{' gpurun_out/fsdp/b2.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); d=j["details"]; print(j["value"], j["ms_per_step"], d.get("comm"), d.get("xgmi_selftest"), (d.get("comm_choice") or {}).get("oneshot_threshold_bytes"))')"
  done
done
grep '^{' gpurun_out/fsdp/b2.log > gpurun_out/fsdp/last_n2.json
unset JDT_BACKEND
timeout -k 10 400 python tools/gemm_split_sweep.py > gpurun_out/fsdp/split_sweep.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/fsdp/split_sweep.txt | sed 's/ | /\n   /g' | head -80
