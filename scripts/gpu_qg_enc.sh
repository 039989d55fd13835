#!/bin/bash
# NGTQG encoder/trainer parity tests, then the qg bench with device quantization.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_qg.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_qg.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_qg.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode qg --no-cpu --steps 6 > gpurun_out/qg_enc.json 2> gpurun_out/qg_enc.log
rc=$?; grep -E "quantizer|eps" gpurun_out/qg_enc.log | tail -4
python -c "
import json;d=json.load(open('gpurun_out/qg_enc.json'));print(round(d['value']),d['config']['recall_at_10'],d['config']['epsilon'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
exit $rc
