set -o pipefail
for d in 0 1 2 4 6; do
  echo "== PBX_TOWER_DEBUG=$d"
  PBX_TOWER_DEBUG=$d timeout -k 10 60 python -u scripts/bench_tower.py --iters 50 2>&1 | grep tower || exit 1
done
