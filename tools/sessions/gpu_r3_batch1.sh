#!/bin/bash
# round 3 batch: every new GPU test, then benches (transformer both modes, FSDP/DP N=2 shared-GPU), then the GEMM split sweep
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/b1
timeout -k 10 900 python -u -m pytest tests/test_reference_loss_fn.py tests/test_lm_gpu.py tests/test_xgmi_gpu.py tests/test_kernels_gpu.py -k "reference or lm_ or fsdp_over_xgmi or xgmi_collectives or ln_gemm or attn128 or transformer or gemm_dropout or dropout" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/b1/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|worst" gpurun_out/b1/pytest.log | tail -40; tail -3 gpurun_out/b1/pytest.log; [ $rc -ne 0 ] && exit $rc
for a in "--strategy pp --model transformer" "--strategy pp --model transformer --microbatch-passes"; do
  for f in 1 0; do
    JDT_LM_FUSED_OPT=$f timeout -k 10 200 python bench.py --steps 200 --warmup 20 $a > gpurun_out/b1/b.log 2>&1 || { tail -3 gpurun_out/b1/b.log; exit 1; }
    echo "'$a' fused_opt=$f: $(grep '^{' gpurun_out/b1/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
export JDT_BACKEND=gloo
for a in "--strategy fsdp" "" "--strategy fsdp --num-layers 4"; do
  for f in 1 0; do
    [ "$a" = "" ] && [ $f -eq 0 ] && continue
    JDT_FSDP_FUSED_COMM=$f timeout -k 10 240 python bench.py --gpus 2 --steps 200 --warmup 20 $a > gpurun_out/b1/b2.log 2>&1 || { tail -5 gpurun_out/b1/b2.log; exit 1; }
    echo "N=2 '$a' fused_comm=$f: $(grep '^{' gpurun_out/b1/b2.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); d=j["details"]; print(j["value"], j["ms_per_step"], d.get("comm"), d.get("xgmi_selftest"), (d.get("comm_choice") or {}).get("oneshot_threshold_bytes"))')"
    grep '^{' gpurun_out/b1/b2.log >> gpurun_out/b1/n2.jsonl
  done
done
unset JDT_BACKEND
timeout -k 10 400 python tools/pp_schedule.py --reps 200 --out gpurun_out/b1/pp_schedule.json > gpurun_out/b1/pp_schedule.log 2>&1 || { tail -20 gpurun_out/b1/pp_schedule.log; exit 1; }
cat gpurun_out/b1/pp_schedule.log
timeout -k 10 400 python tools/gemm_split_sweep.py > gpurun_out/b1/split_sweep.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/b1/split_sweep.txt | sed 's/ | /\n   /g' | head -60
