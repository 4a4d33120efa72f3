# rocprofv3 kernel stats for the secondary BASELINE configs on 1 GPU (one profiled run each).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
i=0
for a in "${@:-"--num-layers 4"}"; do
  i=$((i+1))
  echo "== [$i] $a"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profcfg$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 300 --warmup 30 $a > "$OUT/profcfg$i.log" 2>&1 || { echo "failed rc=$?"; tail -5 "$OUT/profcfg$i.log"; exit 3; }
  grep '^{' "$OUT/profcfg$i.log" | tail -1 | cut -c1-200
done
