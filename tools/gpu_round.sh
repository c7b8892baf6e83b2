#!/bin/bash
# One GPU-box session: parity tests, bench, kernel-trace profile, PMC passes.
# Every GPU step has its own time limit; the first failure ends the script.
# Usage (from the repo root on the box): bash tools/gpu_round.sh [round-tag] [steps...]
set -euo pipefail
TAG=${1:-r01}
shift || true
STEPS=${*:-"test bench prof pmc pmcck pmcrec"}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

for s in $STEPS; do
  case $s in
    test)
      echo "[gpu_round] pytest -m gpu"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
        || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -3 "$OUT/pytest_gpu.log"
      ;;
    smoke)
      echo "[gpu_round] smoke"
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 \
        || { tail -40 "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log"
      ;;
    bench)
      echo "[gpu_round] bench"
      timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" \
        || { tail -40 "$OUT/bench_$TAG.err"; exit 1; }
      cat "$OUT/bench_$TAG.json"
      ;;
    prof)
      echo "[gpu_round] rocprofv3 kernel trace"
      rm -rf "$OUT/prof_$TAG"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o "$TAG" \
        --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-utts 0 --no-north-star \
        > "$OUT/prof_$TAG.log" 2>&1 || { tail -40 "$OUT/prof_$TAG.log"; exit 1; }
      find "$OUT/prof_$TAG" -name '*kernel_stats.csv' -exec cat {} \;
      ;;
    profns)
      echo "[gpu_round] rocprofv3 kernel trace, north-star shape (B=256)"
      rm -rf "$OUT/profns_$TAG"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/profns_$TAG" -o "${TAG}_b256" \
        --output-format csv -- python3 bench.py --batch 256 --steps 10 --warmup 2 --cpu-utts 0 \
        --no-north-star > "$OUT/profns_$TAG.log" 2>&1 || { tail -40 "$OUT/profns_$TAG.log"; exit 1; }
      find "$OUT/profns_$TAG" -name '*kernel_stats.csv' -exec cat {} \;
      ;;
    pmc)
      echo "[gpu_round] PMC passes"
      rm -rf "$OUT/pmc_fetch_$TAG" "$OUT/pmc_write_$TAG"
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$TAG" -o fetch \
        --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-utts 0 \
        --no-north-star > "$OUT/pmc_fetch_$TAG.log" 2>&1 \
        || { tail -40 "$OUT/pmc_fetch_$TAG.log"; exit 1; }
      timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$TAG" -o write \
        --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-utts 0 \
        --no-north-star > "$OUT/pmc_write_$TAG.log" 2>&1 \
        || { tail -40 "$OUT/pmc_write_$TAG.log"; exit 1; }
      python tools/pmc_summary.py --fetch "$OUT/pmc_fetch_$TAG" --write "$OUT/pmc_write_$TAG" \
        --batch 64 --frames 1000 --out "$OUT/${TAG}_pmc_summary_fused.json"
      ;;
    pmcck)
      echo "[gpu_round] PMC passes, checkpointing two-call design"
      rm -rf "$OUT/pmcc_fetch_$TAG" "$OUT/pmcc_write_$TAG"
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmcc_fetch_$TAG" -o fetch \
        --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-utts 0 \
        --no-north-star --design checkpoints > "$OUT/pmcc_fetch_$TAG.log" 2>&1 \
        || { tail -40 "$OUT/pmcc_fetch_$TAG.log"; exit 1; }
      timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmcc_write_$TAG" -o write \
        --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-utts 0 \
        --no-north-star --design checkpoints > "$OUT/pmcc_write_$TAG.log" 2>&1 \
        || { tail -40 "$OUT/pmcc_write_$TAG.log"; exit 1; }
      python tools/pmc_summary.py --fetch "$OUT/pmcc_fetch_$TAG" --write "$OUT/pmcc_write_$TAG" \
        --batch 64 --frames 1000 --out "$OUT/${TAG}_pmc_summary.json"
      ;;
    pmcrec)
      echo "[gpu_round] PMC passes, recursion design"
      rm -rf "$OUT/pmcr_fetch_$TAG" "$OUT/pmcr_write_$TAG"
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmcr_fetch_$TAG" -o fetch \
        --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-utts 0 \
        --no-north-star --design recursion > "$OUT/pmcr_fetch_$TAG.log" 2>&1 \
        || { tail -40 "$OUT/pmcr_fetch_$TAG.log"; exit 1; }
      timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmcr_write_$TAG" -o write \
        --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-utts 0 \
        --no-north-star --design recursion > "$OUT/pmcr_write_$TAG.log" 2>&1 \
        || { tail -40 "$OUT/pmcr_write_$TAG.log"; exit 1; }
      python tools/pmc_summary.py --fetch "$OUT/pmcr_fetch_$TAG" --write "$OUT/pmcr_write_$TAG" \
        --batch 64 --frames 1000 --out "$OUT/${TAG}_pmc_summary_recursion.json"
      ;;
    producer)
      echo "[gpu_round] joint weight function: producer bench, training step, kernel trace"
      rm -rf "$OUT/prodprof_$TAG"
      HS=128,512 timeout -k 10 300 python tools/producer_bench.py > "$OUT/producer_$TAG.jsonl" \
        || { tail -20 "$OUT/producer_$TAG.jsonl"; exit 1; }
      HS=128,512 timeout -k 10 300 python tools/joint_step_bench.py > "$OUT/joint_step_$TAG.jsonl" \
        || { tail -20 "$OUT/joint_step_$TAG.jsonl"; exit 1; }
      HS=512 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prodprof_$TAG" -o prod \
        --output-format csv -- python3 tools/producer_bench.py > "$OUT/prodprof_$TAG.log" 2>&1 \
        || { tail -40 "$OUT/prodprof_$TAG.log"; exit 1; }
      cat "$OUT/producer_$TAG.jsonl" "$OUT/joint_step_$TAG.jsonl"
      ;;
    *)
      echo "unknown step $s"; exit 2;;
  esac
done
echo "[gpu_round] done"
