# ad-hoc GPU batch (the current experiment); see run.sh for the standing tasks
bash scripts/gpu/run.sh sk6 tier smoke bench awq
