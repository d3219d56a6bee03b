bash scripts/gpu/run.sh r6x tier smoke bench ptimeline
