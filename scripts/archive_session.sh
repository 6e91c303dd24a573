#!/bin/bash
# Copy a finished GPU session's gpurun_out/ into profiles/r06/<session>/ (logs,
# CSV summaries; not the raw kernel traces), then clear gpurun_out/ for the next call.
set -eu
cd "$(dirname "$0")/.."
dst=profiles/r06/$1
mkdir -p "$dst"
( cd gpurun_out && find . -type f \( -name "*.log" -o -name "*stats.csv" -o -name "*.json" -o -name "*.txt" \) \
    ! -name ".last_call.json" -print0 | xargs -0 -I{} cp --parents {} "../$dst/" )
rm -rf gpurun_out/*
ls -R "$dst" | head -40
