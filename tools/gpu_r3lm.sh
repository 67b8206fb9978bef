#!/bin/bash
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r3l.sh
bash tools/gpu_r3m.sh
