"""Pure-Python restatement of the reference's concrete opcode arithmetic (test-only).

Each function restates the z3 term the reference builds for an all-concrete stack,
i.e. what ``simplify`` folds it to (mythril/laser/ethereum/instructions.py).
Used to pin the C oracle on random operands; Python ints are the independent
third implementation (oracle: 4x64-bit limbs, device: 8x32-bit limbs).
"""
M = (1 << 256) - 1
T255 = 1 << 255


def s(x):  # two's complement view
    return x - (1 << 256) if x & T255 else x


def z_udiv(a, b):  # bvudiv, x/0 = 2^256-1
    return M if b == 0 else a // b


def z_urem(a, b):  # bvurem, x%0 = x
    return a if b == 0 else a % b


def z_sdiv(a, b):  # bvsdiv (truncating), x/0 = (x<0 ? 1 : -1)
    if b == 0:
        return 1 if s(a) < 0 else M
    q = abs(s(a)) // abs(s(b))
    return (-q if (s(a) < 0) != (s(b) < 0) else q) & M


def z_srem(a, b):  # bvsrem (sign of dividend), x%0 = x
    if b == 0:
        return a
    r = abs(s(a)) % abs(s(b))
    return (-r if s(a) < 0 else r) & M


def signextend(s0, s1):  # instructions.py:640-668, signed s0 <= 31
    testbit = (s0 * 8 + 7) & M
    set_tb = (1 << testbit) & M if testbit < 256 else 0
    sign = (s1 & set_tb) != 0
    if s(s0) <= 31:
        return (s1 | ((0 - set_tb) & M)) if sign else (s1 & ((set_tb - 1) & M))
    return s1


def byte(i, x):  # instructions.py:426-456
    return (x >> ((31 - i) * 8)) & 0xFF if i <= 31 else 0


def sar(value, shift):
    return (s(value) >> min(shift, 256)) & M


# op byte -> (number of operands popped, function of operands in pop order)
BINOPS = {
    0x01: (2, lambda a, b: (a + b) & M),
    0x02: (2, lambda a, b: (a * b) & M),
    0x03: (2, lambda a, b: (a - b) & M),
    0x04: (2, lambda a, b: 0 if b == 0 else z_udiv(a, b)),           # :505-520
    0x05: (2, lambda a, b: 0 if b == 0 else z_sdiv(a, b)),           # :522-537
    0x06: (2, lambda a, b: 0 if b == 0 else z_urem(a, b)),           # :539-551
    0x07: (2, lambda a, b: 0 if b == 0 else z_srem(a, b)),           # :580-592
    0x08: (3, lambda a, b, n: z_urem((z_urem(a, n) + z_urem(b, n)) & M, n)),  # :594-607
    0x09: (3, lambda a, b, n: z_urem((z_urem(a, n) * z_urem(b, n)) & M, n)),  # :609-622
    0x0A: (2, lambda a, b: pow(a, b, 1 << 256)),                      # :624-638
    0x0B: (2, signextend),
    0x10: (2, lambda a, b: int(a < b)),
    0x11: (2, lambda a, b: int(a > b)),
    0x12: (2, lambda a, b: int(s(a) < s(b))),
    0x13: (2, lambda a, b: int(s(a) > s(b))),
    0x14: (2, lambda a, b: int(a == b)),
    0x15: (1, lambda a: int(a == 0)),
    0x16: (2, lambda a, b: a & b),
    0x17: (2, lambda a, b: a | b),
    0x18: (2, lambda a, b: a ^ b),
    0x19: (1, lambda a: M - a),
    0x1A: (2, byte),
    0x1B: (2, lambda sh, v: (v << sh) & M if sh < 256 else 0),
    0x1C: (2, lambda sh, v: v >> sh if sh < 256 else 0),
    0x1D: (2, lambda sh, v: sar(v, sh)),
}


def op_program(op: int, nargs: int) -> bytes:
    """Code that loads nargs operands from calldata (operand k at 32*k, operand 0
    on top), applies `op`, stores the result in slot 0 and stops."""
    code = bytearray()
    for k in reversed(range(nargs)):
        code += bytes([0x60, 32 * k, 0x35])          # PUSH1 32k CALLDATALOAD
    code += bytes([op, 0x60, 0x00, 0x55, 0x00])      # OP PUSH1 0 SSTORE STOP
    return bytes(code)


def special_words():
    return [0, 1, 2, 3, 7, 8, 31, 32, 33, 255, 256, 257, T255, T255 - 1, M, M - 1,
            (1 << 128), (1 << 128) - 1, (1 << 64), 1 << 160, (1 << 160) - 1,
            4 * (1 << 253) + 5, 7 * (1 << 253) + 31, 5 * (1 << 253)]
