"""Extract the RFC 9001 / RFC 9369 Appendix-A vectors that the reference's
tests/test_crypto_v1.py and tests/test_crypto_v2.py hold, into
tests/golden/rfc_vectors.json.

The reference test files are parsed as text with ``ast`` (nothing of the
reference is imported or executed).  Only the literal hex constants and the
numeric packet numbers are kept: they are RFC data, not reference code.

Run once in the build container (needs /root/reference):
    python tests/golden/make_rfc_vectors.py
"""

import ast
import binascii
import json
import os

REF = "/root/reference/tests"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rfc_vectors.json")


def _eval(node, env):
    """Evaluate the tiny expression subset used by the constants."""
    if isinstance(node, ast.Constant):
        return node.value
    if isinstance(node, ast.Call) and getattr(node.func, "attr", None) == "unhexlify":
        return binascii.unhexlify(_eval(node.args[0], env))
    if isinstance(node, ast.Call) and getattr(node.func, "id", None) == "bytes":
        return bytes(_eval(node.args[0], env))
    if isinstance(node, ast.BinOp) and isinstance(node.op, ast.Add):
        return _eval(node.left, env) + _eval(node.right, env)
    if isinstance(node, ast.Name) and node.id in env:
        return env[node.id]
    raise ValueError(ast.dump(node))


def constants(path):
    env = {}
    tree = ast.parse(open(path).read())
    for st in tree.body:
        if isinstance(st, ast.Assign) and len(st.targets) == 1:
            name = getattr(st.targets[0], "id", None)
            if name and name.isupper() and name != "PROTOCOL_VERSION":
                try:
                    env[name] = _eval(st.value, env)
                except ValueError:
                    pass
    return env


def literals_per_test(path):
    """{test method: [hex literals passed to unhexlify inside it, in source order]}"""
    out = {}
    for node in ast.walk(ast.parse(open(path).read())):
        if isinstance(node, ast.FunctionDef) and node.name.startswith(("test_", "create_")):
            lits = []
            for sub in ast.walk(node):
                if isinstance(sub, ast.Call) and getattr(sub.func, "attr", None) == "unhexlify":
                    a = sub.args[0]
                    if isinstance(a, ast.Constant) and isinstance(a.value, str):
                        lits.append((sub.lineno, sub.col_offset, a.value))
            if lits:
                out[node.name] = [v for _, _, v in sorted(lits)]
    return out


def main():
    doc = {}
    for ver, fname in (("v1", "test_crypto_v1.py"), ("v2", "test_crypto_v2.py")):
        env = constants(os.path.join(REF, fname))
        doc[ver] = {
            k: (v.hex() if isinstance(v, bytes) else v) for k, v in sorted(env.items())
        }
        doc[ver]["_literals"] = literals_per_test(os.path.join(REF, fname))
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
