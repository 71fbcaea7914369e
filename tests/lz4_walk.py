"""TEST INFRASTRUCTURE ONLY: a pure-Python walk of an LZ4 block that names the
first rule a block breaks (tests/test_lz4.py uses it to label the few blocks
liblz4 accepts and this repo rejects: a match with offset 0)."""


def first_violation(block: bytes, ulen: int):
    ip = op = 0
    n = len(block)
    while True:
        if ip >= n:
            return "input ends before a token"
        tok = block[ip]; ip += 1
        lit = tok >> 4
        if lit == 15:
            while True:
                if ip >= n:
                    return "literal length past input"
                b = block[ip]; ip += 1; lit += b
                if b != 255:
                    break
        if lit > n - ip or lit > ulen - op:
            return "literals past input or output"
        if op + lit + 12 > ulen or ip + lit + 8 > n:
            if ip + lit != n:
                return "last literals not at input end"
            return None if op + lit == ulen else "short output"
        ip += lit; op += lit
        off = block[ip] | (block[ip + 1] << 8); ip += 2
        if off == 0:
            return "offset 0"
        if off > op:
            return "offset past output"
        ml = (tok & 15) + 4
        if (tok & 15) == 15:
            while True:
                if ip >= n:
                    return "match length past input"
                b = block[ip]; ip += 1; ml += b
                if b != 255 or ml > ulen:
                    break
        if ml + 5 > ulen - op:
            return "match into the last 5 bytes"
        op += ml
