#!/bin/bash
# GPU box, round-3 end: PMC passes over k_cook / k_decook (scripts/pmc_cook.sh)
# on the slicing-by-16, two-chain build, then a per-kernel summary.
bash scripts/pmc_cook.sh && python3 scripts/pmc_summary.py gpurun_out/pmc_cook k_cook k_decook > gpurun_out/pmc_cook/summary.txt 2>&1; cat gpurun_out/pmc_cook/summary.txt | head -40
