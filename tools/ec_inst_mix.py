#!/usr/bin/env python3
"""VALU instruction mix of the generated eval_check kernels, from the built objects
(build/obj/gen__<c>__eval_check_<c>_k*.hip.o): the gfx950 code object is unbundled and
disassembled, and each kernel's VALU instructions are counted in the template instance the
bench runs (k<i><true>, PMC name ec_<c>::k<i><true>). The kernels are straight-line code (one
lane per point, a single bounds branch), so the static count is the per-wave dynamic count;
it is checked against PMC SQ_INSTS_VALU per wave when a valu summary is given.

Each mnemonic gets two issue costs:
  cycles  the guide's wave64 issue cost on a SIMD-32 (MI355X_MICROARCH.md:54): 2 cycles for
          full-rate 32-bit VOP1/VOP2 ops, 4 for the rest (64-bit, multiply, VOP3-only);
  rate    the chip rate measured for that instruction alone at 4 waves per SIMD
          (tools/micro/valu_rates.hip, profiles/archive/r1_valu_rates.txt), T lane-instr/s.
bench.py quotes eval_check's launch against both (roofline.eval_check_issue).

  python tools/ec_inst_mix.py rv32im [profiles/rN_pmc_valu.json] > profiles/rN_ec_inst_mix.json
"""
import glob
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# measured chip rates (T lane-instructions/s, 4 waves per SIMD): r1_valu_rates.txt
MEASURED = {"v_add_u32": 50.55, "v_min_u32": 33.76, "v_mul_lo_u32": 30.40, "v_mul_hi_u32": 33.53,
            "v_mad_u64_u32": 29.26, "v_lshl_add_u64": 31.27, "v_add_co_u32": 31.69, "v_sub_u32": 52.52,
            "v_add3_u32": 33.99}
# full-rate (2-cycle) 32-bit ALU ops; everything else is priced at 4 cycles
FULL_RATE = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_mov_b32", "v_and_b32", "v_or_b32", "v_xor_b32",
             "v_lshlrev_b32", "v_lshrrev_b32", "v_min_u32", "v_max_u32", "v_cndmask_b32"}


def rate_of(m):
    """measured rate of a mnemonic, else the measured rate of its class"""
    if m in MEASURED:
        return MEASURED[m]
    if m in FULL_RATE and m != "v_min_u32":
        return MEASURED["v_add_u32"]  # VOP2 full-rate ops measured at the add/sub rate
    return MEASURED["v_lshl_add_u64"]  # other VOP3 / 64-bit ops: the 4-cycle class


def mix_of_object(obj, kernel_re):
    """{symbol: {mnemonic: count}} of the VALU instructions of each matching kernel symbol"""
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fatbin"), os.path.join(td, "co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(td, "x")])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        dis = subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], text=True)
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1) if re.search(kernel_re, m.group(1)) else None
            if cur:
                out[cur] = {}
            continue
        if cur:
            m = re.match(r"^\s+(v_\w+)", line)
            if m:
                mn = re.sub(r"_e(32|64)$", "", m.group(1))
                out[cur][mn] = out[cur].get(mn, 0) + 1
    return out


def main(circuit, pmc=None):
    objs = sorted(glob.glob(os.path.join(ROOT, "build", "obj", f"gen__{circuit}__eval_check_{circuit}_k*.hip.o")),
                  key=lambda p: int(re.search(r"_k(\d+)\.hip\.o$", p).group(1)))
    pmc_k = json.load(open(pmc))["kernels"] if pmc else {}
    per = {}
    for o in objs:
        k = int(re.search(r"_k(\d+)\.hip\.o$", o).group(1))
        # the template instance the bench runs: the one the PMC pass saw, else <true>
        variant = "false" if f"ec_{circuit}::k{k}<false>" in pmc_k else "true"
        syms = mix_of_object(o, rf"_ZN2r0\d+ec_{circuit}\d+k{k}ILb{1 if variant == 'true' else 0}E")
        assert len(syms) == 1, (o, list(syms))
        per[k] = (variant, next(iter(syms.values())))
    with open(os.path.join(ROOT, "risc0_amd", "lib", "libr0hip.so"), "rb") as f:
        lib = hashlib.sha256(f.read()).hexdigest()[:16]
    kernels = {}
    for k, (variant, mix) in per.items():
        n = sum(mix.values())
        cyc = sum(c * (2 if m in FULL_RATE else 4) for m, c in mix.items())
        lane_s = sum(c * 64 / (rate_of(m) * 1e12) for m, c in mix.items())  # seconds per wave at the chip rate
        d = {"valu_per_wave": n, "issue_cycles_per_wave": cyc, "full_rate_share": round(
            sum(c for m, c in mix.items() if m in FULL_RATE) / max(n, 1), 4),
             "measured_rate_s_per_wave": lane_s, "mix": dict(sorted(mix.items(), key=lambda kv: -kv[1]))}
        d["variant"] = variant
        p = pmc_k.get(f"ec_{circuit}::k{k}<{variant}>")
        if p and p["waves"]:
            d["pmc_valu_per_wave"] = round(p["insts_valu"] / p["waves"], 1)
        kernels[f"k{k}"] = d
    tot = sum(d["valu_per_wave"] for d in kernels.values())
    json.dump({"circuit": circuit, "lib_sha256_16": lib, "source": "tools/ec_inst_mix.py over build/obj",
               "valu_per_point": tot, "issue_cycles_per_point": sum(d["issue_cycles_per_wave"] for d in kernels.values()),
               "measured_rate_s_per_wave": sum(d["measured_rate_s_per_wave"] for d in kernels.values()),
               "kernels": kernels}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
