cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ppa
val() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["details"]["final_loss"])'; }
for st in "5 3" "20 5" "60 10"; do set -- $st
  for ah in 0 1; do
    JDT_MLP2_AHEAD=$ah timeout -k 10 120 python bench.py --strategy pp --hidden-layers 8 --steps $1 --warmup $2 > gpurun_out/ppa/b.log 2>&1 || exit 1
    echo "steps=$1 warmup=$2 ahead=$ah: $(val gpurun_out/ppa/b.log)"
  done
done
for ah in 0 1; do
  JDT_MLP2_AHEAD=$ah timeout -k 10 120 python bench.py --num-layers 4 --steps 60 --warmup 10 > gpurun_out/ppa/b.log 2>&1 || exit 1
  echo "dp4 60 ahead=$ah: $(val gpurun_out/ppa/b.log)"
done
