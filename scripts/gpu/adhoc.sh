bash scripts/gpu/run.sh r6y tier smoke
