"""Parse tests/golden/crc32c_kat.txt (RFC 3720 §B.4 vectors)."""
import os

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "crc32c_kat.txt")


def vectors():
    out = []
    for line in open(PATH):
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        name, spec, exp = line.split()
        if spec == "-":
            data = b""
        elif spec.startswith("zeros:"):
            data = bytes(int(spec[6:]))
        elif spec.startswith("ones:"):
            data = b"\xff" * int(spec[5:])
        elif spec.startswith("inc:"):
            data = bytes(range(int(spec[4:])))
        elif spec.startswith("dec:"):
            data = bytes(range(int(spec[4:]) - 1, -1, -1))
        else:
            data = bytes.fromhex(spec)
        out.append((name, data, int(exp, 16)))
    return out
