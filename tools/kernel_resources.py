"""Per-kernel resource usage of the built gfx950 code objects (scratch bytes, VGPR / SGPR spills, VGPRs, LDS).

The fat-binary section of every object under textmae-image-compression_amd/lib/obj is unbundled with the ROCm LLVM
tools and the code object's metadata notes (.amdhsa.kernels) are read.  A kernel with private-segment bytes spills or
indexes a local array through scratch: on the hot kernels that is a regression (lic_stack_kernel's forward fell
10.1k -> 9.3k img/s when a route field spilled SGPRs).
    python tools/kernel_resources.py [--scratch-only] [substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "textmae-image-compression_amd", "lib", "obj")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FIELDS = ("name", "private_segment_fixed_size", "group_segment_fixed_size", "vgpr_count", "agpr_count",
          "sgpr_count", "vgpr_spill_count", "sgpr_spill_count")


def tools_present():
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf"))


def kernels(obj):
    """[{field: value}] for every kernel of one host object's gfx950 code object"""
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "co.o")
        r = subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", obj, os.devnull],
                           capture_output=True)
        if r.returncode != 0 or not os.path.exists(fb):
            return []  # host-only object (no device code)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", f"--targets={TARGET}",
                        f"--input={fb}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s+-?\s*\.(\w+):\s+(\S+)", line)
        if not m or m.group(1) not in FIELDS:
            continue
        k, v = m.group(1), m.group(2)
        if k in cur:  # the field repeats: next kernel
            out.append(cur)
            cur = {}
        cur[k] = v if k == "name" else int(v)
    if cur:
        out.append(cur)
    return [k for k in out if "name" in k]


def all_kernels():
    res = {}
    for f in sorted(os.listdir(OBJ)):
        if f.endswith(".o"):
            res[f] = kernels(os.path.join(OBJ, f))
    return res


def demangle(names):
    for tool in (os.path.join(LLVM, "llvm-cxxfilt"), "c++filt"):
        try:
            r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True)
        except OSError:
            continue
        if r.returncode == 0:
            return r.stdout.splitlines()
    return list(names)


if __name__ == "__main__":
    args = sys.argv[1:]
    scratch_only = "--scratch-only" in args
    subs = [a for a in args if not a.startswith("--")]
    for obj, ks in all_kernels().items():
        ks = [k for k in ks if (not scratch_only or k.get("private_segment_fixed_size", 0))
              and (not subs or any(s in k["name"] for s in subs))]
        for k, dn in zip(ks, demangle([k["name"] for k in ks])):
            print(f"{obj:22s} scratch {k.get('private_segment_fixed_size', 0):4d}  vgpr {k.get('vgpr_count', 0):3d}  "
                  f"agpr {k.get('agpr_count', 0):3d}  vspill {k.get('vgpr_spill_count', 0):3d}  "
                  f"sspill {k.get('sgpr_spill_count', 0):3d}  lds {k.get('group_segment_fixed_size', 0):6d}  {dn[:120]}")
