"""rv32im BigInt cycles for the accumulation tests (test infrastructure only).

* `states(mix, records)`: BigIntAccum restated over Python integers
  (risc0/circuit/rv32im/src/prove/witgen/byte_poly.rs:381-470): the accumulator state after
  each Back::BigInt record, as the 12 Montgomery words WitnessGenerator::accum scatters into
  accum columns 0..11 (witgen/mod.rs:178-205).
* `program(rng)`: the BigInt cycles of one precompile call whose EqZero checks hold for every
  mix, so the reference accepts them: an ecall row (Reset), then the byte-polynomial program
  of a small integer identity, then the closing Reset (witgen/bigint.rs:97-183 emits rows in
  that shape). Three kinds cover all seven PolyOps: an addition a + b = c with its carries
  (AddTotal, Carry1, Carry2, EqZero), a product a * b = c (SetTerm, AddTotal, carries,
  EqZero), and terms that cancel (Shift, SetTerm, AddTotal with every coefficient).
* `lay_out(rng, rows, ...)`: data rows (211 columns) taking instruction arms like
  test_rv32im_accum_ir.rows_for_arms, with the programs' cycles on arm 12 and their
  BigIntState in data columns 29..50 (LAYOUT_TOP.inst_result.arm12.state,
  rv32im/src/zirgen/layout.rs.inc:17098-17118; BigIntState::offsets, bigint.rs:185-211).
"""
import numpy as np

import verifier as V

P = V.P
WIDTH = 16  # BIGINT_WIDTH_BYTES
RESET, SHIFT, SET_TERM, ADD_TOTAL, CARRY1, CARRY2, EQ_ZERO = range(7)  # PolyOp (bigint.rs:62-70)
STATE_COLS = dict(is_ecall=29, mode=30, pc=31, poly_op=32, coeff=33, bytes=34, next_state=50)
SELECTORS = list(range(1, 14))  # instResult._selector[k]._super: data columns 1..13
BIGINT_ARM = 12
BIGINT_STEP, DECODE = 41, 48  # CycleState (rv32im/src/execute/platform.rs:101-131)


def _e(x):
    return V.efp(x)


def states(mix, records):
    """BigIntAccum::new(final mix) then ::step per (row, poly_op, coeff, bytes) record:
    (n, 12) Montgomery words (poly, term, total). Raises ValueError on an EqZero whose goal is
    nonzero ("Invalid eqz in bigint accum", byte_poly.rs:458)."""
    m = [V.dec(w) for w in mix]
    last_mix = tuple(m[-4:])
    powers, cur = [], (1, 0, 0, 0)
    for _ in range(WIDTH + 1):
        powers.append(cur)
        cur = V.emul(cur, last_mix)
    neg_poly = (0, 0, 0, 0)
    for p in powers[:WIDTH]:
        neg_poly = V.eadd(neg_poly, V.emul(p, _e(128)))
    poly, term, total = (0, 0, 0, 0), (1, 0, 0, 0), (0, 0, 0, 0)
    out = np.zeros((len(records), 12), np.uint32)
    for k, (_row, op, coeff, by) in enumerate(records):
        delta = (0, 0, 0, 0)
        for b, p in zip(by, powers[:WIDTH]):
            delta = V.eadd(delta, V.emul(p, _e(int(b))))
        new_poly = V.eadd(poly, delta)
        if op == RESET:
            poly, term, total = (0, 0, 0, 0), (1, 0, 0, 0), (0, 0, 0, 0)
        elif op == SHIFT:
            poly = V.emul(new_poly, powers[WIDTH])
        elif op == SET_TERM:
            poly, term = (0, 0, 0, 0), new_poly
        elif op == ADD_TOTAL:
            c = V.esub(_e(coeff), _e(4))
            total = V.eadd(total, V.emul(V.emul(c, term), new_poly))
            poly, term = (0, 0, 0, 0), (1, 0, 0, 0)
        elif op == CARRY1:
            poly = V.eadd(poly, V.emul(V.esub(delta, neg_poly), _e(64 * 256)))
        elif op == CARRY2:
            poly = V.eadd(poly, V.emul(delta, _e(256)))
        elif op == EQ_ZERO:
            goal = V.eadd(total, V.emul(new_poly, V.esub(powers[1], _e(256))))
            if goal != (0, 0, 0, 0):
                raise ValueError("Invalid eqz in bigint accum")
            poly, term, total = (0, 0, 0, 0), (1, 0, 0, 0), (0, 0, 0, 0)
        else:
            raise ValueError(f"invalid poly_op {op}")
        out[k] = [V.enc(x) for x in poly + term + total]
    return out


def _bytes(v, n=WIDTH):
    return [(v >> (8 * i)) & 0xFF for i in range(n)]


def _carry_rows(coeffs):
    """Carry1, Carry2 and EqZero bytes whose sum (d - 128) * 16384 + e * 256 + f is each
    coefficient of the carry polynomial (Carry1 adds (D - 128 * sum x^i) * 64 * 256, Carry2
    E * 256, EqZero's own bytes F; byte_poly.rs:437-460); coefficients in [-2^21, 2^21)"""
    d, e, f = [], [], []
    for v in list(coeffs) + [0] * (WIDTH - len(coeffs)):
        u = v + 128 * 16384
        assert 0 <= u < 256 * 16384, v
        d.append(u // 16384)
        e.append((u % 16384) // 256)
        f.append(u % 256)
    return [(CARRY1, 4, d), (CARRY2, 4, e), (EQ_ZERO, 4, f)]


def _quotient(p):
    """P(x) / (x - 256) for integer coefficients with P(256) = 0"""
    q = [0] * (len(p) - 1)
    acc = 0
    for i in range(len(p) - 1, 0, -1):
        acc = p[i] + 256 * acc
        q[i - 1] = acc
    assert p[0] + 256 * acc == 0
    return q


def program(rng, kind):
    """(poly_op, coeff, bytes) cycles of one BigInt call; coeff is BigIntState::coeff (+4)"""
    rows = [(RESET, 0, [0] * WIDTH)]  # the ecall cycle (bigint.rs:241-256)
    if kind == "add":  # a + b = c (15-byte operands, so no carry leaves the top byte)
        a, b = (int(rng.integers(0, 1 << 60)) << 60 | int(rng.integers(0, 1 << 60)) for _ in range(2))
        a, b = a % (1 << 120), b % (1 << 120)
        c = a + b
        rows += [(ADD_TOTAL, 5, _bytes(a)), (ADD_TOTAL, 5, _bytes(b)), (ADD_TOTAL, 3, _bytes(c))]
        pc = [x + y - z for x, y, z in zip(_bytes(a), _bytes(b), _bytes(c))]
        rows += _carry_rows([-q for q in _quotient(pc + [0])])
    elif kind == "mul":  # a * b = c (8-byte operands)
        a, b = (int(rng.integers(0, 1 << 62)) * 4 + int(rng.integers(0, 4)) for _ in range(2))
        c = a * b
        rows += [(SET_TERM, 4, _bytes(a)), (ADD_TOTAL, 5, _bytes(b)), (ADD_TOTAL, 3, _bytes(c))]
        pa, pb, pcc = _bytes(a), _bytes(b), _bytes(c)
        prod = [0] * (2 * WIDTH)
        for i, x in enumerate(pa):
            for j, y in enumerate(pb):
                prod[i + j] += x * y
        pc = [prod[i] - (pcc[i] if i < WIDTH else 0) for i in range(2 * WIDTH)]
        while len(pc) > WIDTH + 1:
            assert pc[-1] == 0
            pc.pop()
        rows += _carry_rows([-q for q in _quotient(pc)])
    elif kind == "cancel":  # T*R - T*R + k*(H x^16 + L) - k*(H x^16 + L) = 0
        t, r, h, l = ([int(v) for v in rng.integers(0, 256, WIDTH)] for _ in range(4))
        k = int(rng.integers(1, 4))  # AddTotal coefficient k and -k: coeff 4 + k, 4 - k
        rows += [(SET_TERM, 4, t), (ADD_TOTAL, 5, r), (SET_TERM, 4, t), (ADD_TOTAL, 3, r),
                 (SHIFT, 4, h), (ADD_TOTAL, 4 + k, l), (SHIFT, 4, h), (ADD_TOTAL, 4 - k, l)]
        rows += _carry_rows([0] * WIDTH)
    else:
        raise ValueError(kind)
    rows.append((RESET, 4, [0] * WIDTH))  # the closing cycle (next_state Decode)
    return rows


def lay_out(rng, rows, n_calls, first_row=1):
    """Data rows (211 x rows, Montgomery words; other cycles take random arms 0..11) and the
    BigInt records [(row, poly_op, coeff, bytes)] of n_calls programs placed at random gaps
    from first_row on."""
    import rv32im_accum_ref as R
    draw = lambda n: rng.integers(1, P, n, dtype=np.uint64).astype(np.uint32)
    data = draw(R.DATA_COLS * rows).reshape(R.DATA_COLS, rows)
    arms = list(rng.integers(0, BIGINT_ARM, rows))
    records, ecalls = [], set()
    row = first_row
    kinds = ["add", "mul", "cancel"]
    for i in range(n_calls):
        prog = program(rng, kinds[i % 3])
        row += int(rng.integers(0, 4))
        if row + len(prog) > rows:
            break
        ecalls.add(row)  # the first cycle of a call is its ecall (is_ecall = 1)
        for k, (op, coeff, by) in enumerate(prog):
            records.append((row + k, op, coeff, by))
        row += len(prog)
    enc = lambda v: V.enc(int(v))
    for r, op, coeff, by in records:
        arms[r] = BIGINT_ARM
        is_ecall = 1 if r in ecalls else 0
        data[STATE_COLS["is_ecall"], r] = enc(is_ecall)
        data[STATE_COLS["mode"], r] = enc(0)
        data[STATE_COLS["pc"], r] = enc(int(rng.integers(0, 1 << 20)) * 4)
        data[STATE_COLS["poly_op"], r] = enc(op)
        data[STATE_COLS["coeff"], r] = enc(coeff)
        for i in range(WIDTH):
            data[STATE_COLS["bytes"] + i, r] = enc(by[i])
        data[STATE_COLS["next_state"], r] = enc(DECODE if (op == RESET and not is_ecall) else BIGINT_STEP)
    for r, a in enumerate(arms):
        data[SELECTORS[:a], r] = 0
    return data.reshape(-1), records


def inject(accum, rows, mix, records):
    """WitnessGenerator::accum's scatter (witgen/mod.rs:187-205) into a column-major accum
    group: accum[col * rows + row] = state word col, col < 12"""
    st = states(mix, records)
    a = accum.reshape(-1, rows)
    for (row, *_), s in zip(records, st):
        a[:12, row] = s
    return accum
