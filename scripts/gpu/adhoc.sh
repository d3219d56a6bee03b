bash scripts/gpu/run.sh r6z tier smoke bench2 awq timeline ptimeline
