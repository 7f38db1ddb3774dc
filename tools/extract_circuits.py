#!/usr/bin/env python3
"""Extract circuit *data* (tap sets, poly-mix power lists, protocol info) from the
reference's generated Rust tables into compact JSON under risc0_amd/circuits/.

Runs in the build container only (reads /root/reference); the JSON it writes is
committed, so nothing at run time needs the reference tree.

Sources (reference @ /root/reference):
  rv32im    : risc0/circuit/rv32im/src/zirgen/taps.rs, zirgen/info.rs, zirgen/defs.rs.inc
  recursion : risc0/circuit/recursion/src/taps.rs, src/info.rs
The TapSet semantics follow risc0/zkp/src/taps.rs:57-140.
"""
import json
import os
import re
import sys

REF = os.environ.get("R0_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "risc0_amd", "circuits")


def _ints(s):
    return [int(x) for x in re.findall(r"\d+", s)]


def parse_tapset(path):
    src = open(path).read()
    taps = []
    for m in re.finditer(r"TapData\s*\{([^}]*)\}", src):
        body = m.group(1)
        fields = dict(re.findall(r"(\w+)\s*:\s*(\d+)", body))
        taps.append([int(fields["offset"]), int(fields["back"]), int(fields["group"]),
                     int(fields["combo"]), int(fields["skip"])])

    def arr(name):
        m = re.search(name + r"\s*:\s*&\[([^\]]*)\]", src)
        return _ints(m.group(1))

    def scalar(name):
        return int(re.search(name + r"\s*:\s*(\d+)", src).group(1))

    names = re.findall(r'"(\w+)"', re.search(r"group_names\s*:\s*&\[([^\]]*)\]", src).group(1))
    return {
        "taps": taps,
        "combo_taps": arr("combo_taps"),
        "combo_begin": arr("combo_begin"),
        "group_begin": arr("group_begin"),
        "combos_count": scalar("combos_count"),
        "reg_count": scalar("reg_count"),
        "tot_combo_backs": scalar("tot_combo_backs"),
        "group_names": names,
    }


def parse_info(path):
    src = open(path).read()
    info = re.search(r'ProtocolInfo\(\*b"([^"]*)"\)', src).group(1)
    out_size = int(re.search(r"OUTPUT_SIZE\s*:\s*usize\s*=\s*(\d+)", src).group(1))
    mix_size = int(re.search(r"MIX_SIZE\s*:\s*usize\s*=\s*(\d+)", src).group(1))
    pows = _ints(re.search(r"POLY_MIX_POWERS\s*:\s*&\[usize\]\s*=\s*&\[([^\]]*)\]", src).group(1))
    return info, out_size, mix_size, pows


def build(name, taps_rs, info_rs, group_order, eval_args):
    ts = parse_tapset(taps_rs)
    info, out_size, mix_size, pows = parse_info(info_rs)
    # group sizes (TapSet::group_size, taps.rs:100-104)
    sizes = []
    for g in range(len(ts["group_names"])):
        last = ts["taps"][ts["group_begin"][g + 1] - 1][0]
        sizes.append(last + 1)
    ts.update({
        "name": name,
        "circuit_info": info,
        "output_size": out_size,
        "mix_size": mix_size,
        "poly_mix_powers": pows,
        "group_sizes": sizes,
        # order of the buffers handed to poly_fp(args[]) by the circuit's eval_check
        "eval_args": eval_args,
    })
    assert len(ts["taps"]) == ts["group_begin"][-1], (len(ts["taps"]), ts["group_begin"])
    return ts


def main():
    os.makedirs(OUT, exist_ok=True)
    c = os.path.join(REF, "risc0", "circuit")
    circuits = {
        # rv32im: args = [accum, data, out(global), mix]   (rv32im/src/prove/hal/cpu.rs:177)
        "rv32im": build("rv32im",
                        os.path.join(c, "rv32im/src/zirgen/taps.rs"),
                        os.path.join(c, "rv32im/src/zirgen/info.rs"),
                        None, ["accum", "data", "global", "mix"]),
        # recursion: args = [ctrl(code), global, data, mix, accum] (recursion-sys/kernels/cxx/ffi.cpp:225-231)
        "recursion": build("recursion",
                           os.path.join(c, "recursion/src/taps.rs"),
                           os.path.join(c, "recursion/src/info.rs"),
                           None, ["code", "global", "data", "mix", "accum"]),
    }
    for name, d in circuits.items():
        path = os.path.join(OUT, name + ".taps.json")
        with open(path, "w") as f:
            json.dump(d, f, separators=(",", ":"))
        print(f"{name}: {len(d['taps'])} taps, groups {d['group_names']} sizes {d['group_sizes']}, "
              f"combos {d['combos_count']}, regs {d['reg_count']}, poly_mix {len(d['poly_mix_powers'])} -> {path}")


if __name__ == "__main__":
    sys.exit(main())
