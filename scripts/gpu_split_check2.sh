#!/bin/bash
# GPU box: run-time (hipRTC) split-k networks: RTC tests, encode parity, bench line, probe.
export RSMI_RTC_CACHE=$PWD/gpurun_out/rtc_cache
timeout -k 10 500 python -u -m pytest tests/test_bitslice_rtc.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "rtc or encode or c1 or concurrent" > gpurun_out/split2_tests.log 2>&1 || { tail -30 gpurun_out/split2_tests.log; exit 1; }
tail -2 gpurun_out/split2_tests.log
rm -rf gpurun_out/rtc_cache
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/split2_bench.json 2> gpurun_out/split2_bench.err || { tail gpurun_out/split2_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/split2_bench.json')); print(d['value'], d['encode_ms'], d['decode_ms'], d['roofline']['frac'], d['other_configs']['rtc_f10_5_encode'])"
timeout -k 10 120 scripts/probes/mix_probe > gpurun_out/mix_probe4.txt 2>&1 && grep -E 'split|again' gpurun_out/mix_probe4.txt
