#!/bin/bash
# Build an experimental variant of the library: scripts/build_exp.sh NAME "-DFOO=1 -DBAR=2" [KERNELS_SRC]
# -> frender_amd/libfrender_hip_exp_NAME.so (objects in build/exp_NAME; only changed sources recompile).
# KERNELS_SRC: another fr_kernels.hip (e.g. a git revision's, written to build/): A/B against the tree.
set -eu
cd "$(dirname "$0")/.."
python3 - "$1" "${2:-}" "${3:-}" <<'PY'
import os, shlex, sys
sys.path.insert(0, os.getcwd())
import __graft_entry__ as g
name, flags, ksrc = sys.argv[1], shlex.split(sys.argv[2]), sys.argv[3]
srcs = [os.path.abspath(ksrc) if ksrc and os.path.basename(s) == "fr_kernels.hip" else s for s in g.SOURCES]
g.build_lib(flags=flags, out=os.path.join(g.PKG, f"libfrender_hip_exp_{name}.so"),
            objdir=os.path.join(g.ROOT, "build", f"exp_{name}"), sources=srcs)
PY
