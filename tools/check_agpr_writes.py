"""Build-time guard for the four-wave GEMM objects (gemm_g4.o): their main loop is one inline-
assembly block that owns a0-a255 (the accumulators), and the epilogue reads them back in later asm
statements. That only works if the compiler never puts a value of its own into an AGPR between
those statements (an AGPR spill slot, a register-class copy). This script disassembles the object's
gfx950 code and refuses it when any instruction writes an AGPR other than the asm block's own
writes: `v_accvgpr_write_b32 aN, 0` (zeroing) and the MFMAs (accumulation).

  python3 tools/check_agpr_writes.py multimodal-misinformation-detection_amd/csrc/build/gemm_g4.o
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
AGPR = re.compile(r"^a(\d+|\[\d+:\d+\])$")
# instructions whose first operand is a SOURCE (data of a store / DMA), not a destination
SRC_FIRST = ("buffer_store", "global_store", "flat_store", "scratch_store", "ds_write", "ds_store")


def device_code(obj, tmp):
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(tmp, "host.o")],
                   check=True)
    co = os.path.join(tmp, "dev.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"], check=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                          capture_output=True, text=True).stdout


def bad_writes(asm):
    bad, fn = [], "?"
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            fn = m.group(1)
            continue
        ins = line.split("//")[0].strip()
        if not ins or not ins[0].isalpha():
            continue
        parts = ins.replace(",", " ").split()
        op = parts[0]
        if len(parts) < 2 or op.startswith(SRC_FIRST) or not AGPR.match(parts[1]):
            continue
        if op.startswith("v_mfma"):
            continue
        if op == "v_accvgpr_write_b32" and len(parts) == 3 and parts[2] == "0":
            continue
        bad.append(f"{fn}: {ins}")
    return bad


def main(objs):
    rc = 0
    for obj in objs:
        with tempfile.TemporaryDirectory() as tmp:
            bad = bad_writes(device_code(obj, tmp))
        if bad:
            rc = 1
            print(f"error: {obj}: {len(bad)} compiler-placed AGPR write(s) outside the assembly blocks "
                  f"(the accumulators a0-a255 would be clobbered):", file=sys.stderr)
            for b in bad[:20]:
                print("  " + b, file=sys.stderr)
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
