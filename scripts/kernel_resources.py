"""Scratch (private segment) bytes, VGPRs and spills of the kernels in a built object
(scripts only): extracts the gfx950 code object from build/<name>.o and reads its notes.
usage: python scripts/kernel_resources.py [tiled] [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

obj = sys.argv[1] if len(sys.argv) > 1 else "tiled"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
o = os.path.join(root, "vaex_amd", "csrc", "build", obj + ".o")
llvm = "/opt/rocm/lib/llvm/bin/"
with tempfile.TemporaryDirectory() as d:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
    subprocess.run([llvm + "llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, o], check=True)
    subprocess.run([llvm + "clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
    notes = subprocess.run([llvm + "llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
for b in re.split(r"\n\s+- \.agpr_count", notes):
    m = re.search(r"\.name:\s+(\S+)", b)
    if not m or flt not in m.group(1):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", b) or [None, "?"])[1]
    dm = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
    print(f"scratch {g('private_segment_fixed_size'):>5}  vgpr {g('vgpr_count'):>4}  spill {g('vgpr_spill_count'):>3}  {dm[:110]}")
