#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 700 bash scripts/gpu_r05_f.sh && timeout -k 10 400 bash scripts/gpu_r05_d.sh
