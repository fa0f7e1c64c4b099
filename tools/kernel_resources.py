"""Per-kernel VGPR / scratch / spill counts of every gfx950 code object inside a built library (all translation units
of the .hip_fatbin section). Used by tests/test_abi.py (no kernel may spill VGPRs: DESIGN.md section 4, "Skewed keys")
and from the command line: python tools/kernel_resources.py [library] [name-regexp]."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernels(lib):
    """[{name, vgpr_count, vgpr_spill_count, sgpr_spill_count, private_segment_fixed_size}] over all code objects."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, lib,
                               os.path.join(d, "x.so")])
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            part = os.path.join(d, "b%d.bin" % i)
            open(part, "wb").write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, "co%d.o" % i)
            r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + part,
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], capture_output=True)
            if r.returncode or not os.path.getsize(co):
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True,
                                   text=True).stdout
            cur = None
            for line in notes.splitlines():
                m = re.match(r"\s*\.name:\s+(\S+)", line)
                if m:
                    cur = {"name": m.group(1)}
                    out.append(cur)
                    continue
                m = re.match(r"\s*\.(vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size):\s+(\d+)",
                             line)
                if m and cur is not None:
                    cur[m.group(1)] = int(m.group(2))
    return [k for k in out if "vgpr_count" in k]


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "flink_amd",
                                                                  "libflink_amd.so")
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    ks = kernels(lib)
    for k in ks:
        if pat.search(k["name"]):
            print("%3d VGPR  %3d VGPR-spill  %3d SGPR-spill  %4d scratch  %s" % (
                k["vgpr_count"], k.get("vgpr_spill_count", 0), k.get("sgpr_spill_count", 0),
                k.get("private_segment_fixed_size", 0), k["name"]))
    print("%d kernels, %d spill VGPRs" % (len(ks), sum(k.get("vgpr_spill_count", 0) > 0 for k in ks)))


if __name__ == "__main__":
    main()
