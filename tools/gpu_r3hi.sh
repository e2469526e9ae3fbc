# r3h (pipelined multi-tile A/B) then r3i (flow slot record: tests + F1 A/B + counter list)
bash tools/gpu_r3h.sh && bash tools/gpu_r3i.sh
