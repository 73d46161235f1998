#!/bin/bash
# Record the fill order of Vec3(f(), f(), f()) (the reference's Random(), Math.cuh:231-234) for the compilers in
# this image: g++ (the survey's host build of the reference), clang (hipcc's host side), and hipcc's gfx950
# device compile — statically from its LLVM IR here, and by running it when a GPU is present (RUN_DEVICE=1).
# Output: one line per compiler, e.g. into profiles/r05_fill_order.txt.
set -eu
cd "$(dirname "$0")"
out=${OUT_DIR:-../../build/fill_order}
mkdir -p "$out"
g++ -O2 -o "$out/host_gxx" probe_host.cpp && echo "g++ $(g++ -dumpversion) -O2 host: $("$out/host_gxx")"
g++ -O0 -o "$out/host_gxx0" probe_host.cpp && echo "g++ $(g++ -dumpversion) -O0 host: $("$out/host_gxx0")"
/opt/rocm/llvm/bin/clang++ -O2 -o "$out/host_clang" probe_host.cpp && echo "clang++ (ROCm) -O2 host: $("$out/host_clang")"
# device IR at -O0: the calls to draw() stay calls, in evaluation order; record the order of the three stores
# each call's result makes into the constructor's arguments
/opt/rocm/bin/hipcc --offload-arch=gfx950 --cuda-device-only -O0 -emit-llvm -S -o "$out/probe_device.ll" probe_device.hip
python3 - "$out/probe_device.ll" <<'PY'
import re, sys
ir = open(sys.argv[1]).read()
body = ir[ir.index("define"):]
fn = re.search(r"define [^\n]*random_vec[^\n]*\{(.*?)\n\}", ir, re.S)
calls = re.findall(r"(%[\w.]+) = call [^\n]*@_Z4drawP5Draws", fn.group(1))
ctor = re.search(r"call [^\n]*@_ZN5Vec3pC[12]Efff\([^,]+, float ([^,]+), float ([^,]+), float ([^)]+)\)", fn.group(1))
args = [a.strip().split()[-1] for a in ctor.groups()]
order = [calls.index(a) + 1 for a in args]  # the call index (1 = first evaluated) feeding x, y, z
name = "left-to-right" if order == [1, 2, 3] else ("right-to-left" if order == [3, 2, 1] else "other")
print(f"hipcc gfx950 device IR (-O0): x=draw#{order[0]} y=draw#{order[1]} z=draw#{order[2]} -> {name}")
PY
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -o "$out/probe_device" probe_device.hip
if [ "${RUN_DEVICE:-0}" = 1 ]; then timeout -k 5 60 "$out/probe_device"; fi
