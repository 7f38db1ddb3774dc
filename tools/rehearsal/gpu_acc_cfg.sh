# accumulation parity + bench leg, then the other BASELINE configs (tools/gpu_configs.sh)
bash tools/rehearsal/gpu_acc4.sh && bash tools/gpu_configs.sh r2q_configs
