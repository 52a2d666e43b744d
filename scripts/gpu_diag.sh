#!/bin/bash
# Timing diagnosis of the pipelined forward kernel on the GPU box, against the -DFG_F3_DIAG copy
# of the library that `python scripts/gpu_diag.sh build` (on the build host) leaves in
# flood-prediction-gan_amd/build/diag/ (the in-tree product library is left alone).
cd "$(dirname "$0")/.." || exit 1
DIAG=flood-prediction-gan_amd/build/diag
if [ "$1" = "build" ]; then
  python - <<'EOF'
import os, sys
sys.path.insert(0, "flood-prediction-gan_amd")
from floodgan import build as B
d = os.path.join(B.PKG_ROOT, "build", "diag")
B.OBJDIR = os.path.join(d, "obj")
B.LIBDIR = d
B.LIB = os.path.join(d, "libfloodgan.so")
B.build(extra=["-DFG_F3_DIAG"])
EOF
  exit $?
fi
mkdir -p gpurun_out
FLOODGAN_LIB=$PWD/$DIAG/libfloodgan.so timeout -k 10 300 python -u scripts/diag_f3.py "$@" > gpurun_out/diag_f3.log 2>&1
rc=$?; cat gpurun_out/diag_f3.log; exit $rc
