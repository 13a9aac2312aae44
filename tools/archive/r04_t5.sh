#!/bin/bash
set -u
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
