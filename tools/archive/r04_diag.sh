#!/bin/bash
set -u
timeout -k 10 120 python tools/archive/diag_rows.py 2>&1 | grep -v amdgpu.ids
