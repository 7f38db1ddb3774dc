"""Big-integer restatement of the Poseidon254 hash suite (test infrastructure only), used
to cross-check the C++ oracle on small inputs. Follows
risc0/zkp/src/core/hash/poseidon_254/mod.rs:
  sbox / full_round / partial_round / poseidon_mix   :33-89
  digest_to_fr / fr_to_digest                        :94-105 (little-endian bytes)
  unpadded_hash (8 BabyBear values per Fr, base p)   :107-133
  hash_pair                                          :136-142
  Poseidon254Rng mix / random_bits / random_elem     :157-209
Elements enter as canonical BabyBear integers (Elem::as_u32)."""
import json
import os

_P = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "poseidon254_params.json")))
MOD = int(_P["modulus"])
RC = [int(x) for x in _P["round_constants"]]
MDS = [int(x) for x in _P["mds"]]
HALF_FULL, PARTIAL = _P["rounds_half_full"], _P["rounds_partial"]
BB = 15 * (1 << 27) + 1


def mix(c):
    r = 0
    for kind in ["f"] * HALF_FULL + ["p"] * PARTIAL + ["f"] * HALF_FULL:
        c = [(c[i] + RC[3 * r + i]) % MOD for i in range(3)]
        n = 3 if kind == "f" else 1
        c = [pow(x, 8, MOD) if i < n else x for i, x in enumerate(c)]
        c = [sum(MDS[3 * i + j] * c[j] for j in range(3)) % MOD for i in range(3)]
        r += 1
    return c


def to_words(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def from_words(w):
    x = sum(int(v) << (32 * i) for i, v in enumerate(w))
    assert x < MOD
    return x


def hash_elems(vals):
    """unpadded_hash over canonical BabyBear values -> digest words"""
    c = [0, 0, 0]
    mul, idx, count = 1, 1, 0
    for v in vals:
        c[idx] = (c[idx] + mul * int(v)) % MOD
        mul = mul * BB % MOD
        count += 1
        if count == 8:
            mul, count, idx = 1, 0, idx + 1
        if idx == 3:
            c = mix(c)
            c[1] = c[2] = 0
            idx = 1
    if idx != 1 or count != 0:
        c = mix(c)
    return to_words(c[0])


def hash_pair(a, b):
    return to_words(mix([0, from_words(a), from_words(b)])[0])


class Rng:
    def __init__(self):
        self.c = [0, 0, 0]

    def mix(self, d):
        self.c[1] = (self.c[1] + from_words(d)) % MOD
        self.c = mix(self.c)

    def random_bits(self, bits):
        src = self.c[2]
        self.c = mix(self.c)
        return src & ((1 << bits) - 1)

    def random_elem(self):
        src = self.c[2]
        self.c = mix(self.c)
        return (src & ((1 << 160) - 1)) % BB
