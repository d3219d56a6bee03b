bash scripts/gpu/run.sh r6w bench
