"""Static checks on the gfx950 code object inside the built libfloodgan.so (no GPU needed).

conv_f3.hip's stage wait (wait_stage) counts the VMEM operations a wave may leave in flight after an epilogue as the
epilogue's store count: NSTV = TM * TN dwordx4 stores on NHWC outputs (one per 16 x 16 block, a lane's 4 consecutive
channels), NSTS = TM * TN * 4 dword stores on strided outputs -- issued unconditionally.  If the compiler ever merged
or split those stores, or dropped some, the count would be too loose and a stage's LDS could be read before its DMA
landed, with no error anywhere.  This test disassembles every conv_fwd_f3_kernel instantiation and checks that it
issues exactly NSTV dwordx4 and NSTS dword buffer stores and no other widths."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "flood-prediction-gan_amd", "floodgan", "lib", "libfloodgan.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else None


def _disassemble(tmp_path):
    """the device disassembly of every bundle in the library's .hip_fatbin section (one bundle per source file)"""
    objcopy, bundler, objdump = _tool("llvm-objcopy"), _tool("clang-offload-bundler"), _tool("llvm-objdump")
    if not (objcopy and bundler and objdump and os.path.exists(LIB)):
        pytest.skip("needs the built library and the ROCm LLVM tools")
    fat = tmp_path / "fat.bin"
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fat}", LIB, str(tmp_path / "host.o")], check=True)
    data = fat.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert offs, "no offload bundle in .hip_fatbin"
    out = []
    for k, o in enumerate(offs):
        b, co = tmp_path / f"b{k}.bin", tmp_path / f"c{k}.o"
        b.write_bytes(data[o:offs[k + 1] if k + 1 < len(offs) else len(data)])
        subprocess.run([bundler, "--unbundle", "--type=o", f"--targets={TARGET}", f"--input={b}", f"--output={co}"],
                       check=True)
        out.append(subprocess.run([objdump, "-d", str(co)], check=True, capture_output=True, text=True).stdout)
    return "\n".join(out)


def _functions(dis):
    for chunk in re.split(r"\n(?=[0-9a-f]+ <[^>]+>:\n)", dis):
        m = re.match(r"[0-9a-f]+ <([^>]+)>:", chunk)
        if m:
            yield m.group(1), chunk


def _demangle(names):
    filt = shutil.which("c++filt")
    if filt is None:
        pytest.skip("needs c++filt")
    res = subprocess.run([filt], input="\n".join(names), check=True, capture_output=True, text=True).stdout
    return res.strip().split("\n")


def test_conv_f3_epilogue_store_count(tmp_path):
    funcs = [(n, body) for n, body in _functions(_disassemble(tmp_path)) if "conv_fwd_f3_kernel" in n]
    assert funcs, "no conv_fwd_f3_kernel in the code object"
    names = _demangle([n for n, _ in funcs])
    checked = 0
    for name, (_, body) in zip(names, funcs):
        m = re.search(r"conv_fwd_f3_kernel<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (true|false), (true|false)(?:, (?:true|false))?>", name)
        assert m, name
        wm, wn = int(m.group(3)), int(m.group(4))
        nstv = (wm // 16) * (wn // 16)
        stores = len(re.findall(r"\bbuffer_store_dword\b", body))
        x4 = len(re.findall(r"\bbuffer_store_dwordx4\b", body))
        other = len(re.findall(r"\bbuffer_store_dwordx[23]\b", body))
        assert other == 0, f"{name}: {other} dwordx2/x3 buffer stores"
        assert x4 == nstv, f"{name}: {x4} dwordx4 buffer stores, wait_stage assumes NSTV = {nstv}"
        assert stores == 4 * nstv, f"{name}: {stores} dword buffer stores, wait_stage assumes NSTS = {4 * nstv}"
        checked += 1
    assert checked >= 12
