#!/bin/bash
# GPU box, round-3 end: cook two-chain A/B (gpu_cook_ab3.sh), then the whole
# suite + smoke (gpu_suite.sh), then bench + kernel trace (gpu_r03_prof.sh final_s4).
bash scripts/gpu_cook_ab3.sh && bash scripts/gpu_suite.sh && NO_PMC=1 bash scripts/gpu_r03_prof.sh final_s4
