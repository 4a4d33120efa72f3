set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s38
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s38
#timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "embedding_fused or xent_metric_slab or embedding_and_colsum or layernorm or ln_gemm or transformer_step" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 3; }
#tail -3 $O/t.log
#timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lm_gpu.py > $O/lm.log 2>&1 || { tail -30 $O/lm.log; exit 3; }
#tail -2 $O/lm.log
for r in 1 2 3; do
  for e in 0 1; do
    JDT_EMBED_LN=$e timeout -k 10 200 python bench.py --strategy pp --model transformer --steps 400 --warmup 40 > $O/b_${e}_${r}.log 2>&1 || { tail -20 $O/b_${e}_${r}.log; exit 3; }
    echo "embed_ln=$e run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${e}_${r}.log)"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_lm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lm.log; exit 3; }
cd $GRAFT_REPO_ROOT; grep -E "metrics_fold|ln_fwd|embed" $O/prof_lm/lm_kernel_stats.csv | cut -c1-160
