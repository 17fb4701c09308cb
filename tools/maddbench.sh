#!/bin/bash
# build tools/maddbench (default product and field code) and run it: tools/maddbench.sh [tag]
set -euo pipefail
cd "$(dirname "$0")/.."
if [ -z "${GRAFT_REPO_ROOT:-}" ]; then
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/maddbench.hip -o tools/maddbench
else
  timeout -k 10 60 tools/maddbench "${1:-lib}"
fi
