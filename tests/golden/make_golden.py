#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the CPU oracle.

PARITY UNPINNED: the fixtures record what the oracle's restatement of ISA-L +
ELECT's coder (oracle/ec_oracle.c) produces.  No run of the reference's
libec.so / ISA-L was possible here (libisal and jni.h are absent; the
reference's erasure_coder.c needs <isa-l.h>), and the reference's own EC test
(ErasureCodeTest.java) holds no vectors.  Each fixture file says so in its
"provenance" field.  The fixtures freeze the oracle so that any later change to
it, or any GPU divergence, shows up as a diff.

Inputs are splitmix64 byte streams (oracle_fill_splitmix: x += 0x9E3779B97F4A7C15,
two xorshift-multiply rounds, little-endian words), keyed per case, so a fixture
is (k, m, L, seeds) -> expected bytes.  Outputs up to 64 bytes are stored in
full (hex); longer ones as SHA-256.

  python tests/golden/make_golden.py   (rewrites the JSON files)
"""
import hashlib
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

from oracle import ec_oracle as o  # noqa: E402
from java_random import JavaRandom  # noqa: E402

PROVENANCE = ("CPU oracle (oracle/ec_oracle.c): restatement of ISA-L's base routines + ELECT's "
              "EC/erasure_coder.c logic. PARITY UNPINNED: not checked against a run of libec.so/ISA-L "
              "(absent from the image; the reference test holds no vectors).")

LENGTHS = [1, 15, 16, 33, 1024, 4099, 65536]
CODES = [(4, 2), (8, 4), (2, 2), (3, 2), (4, 1), (10, 4)]


def seed_of(*parts) -> int:
    h = hashlib.sha256(("/".join(str(p) for p in parts)).encode()).digest()
    return int.from_bytes(h[:8], "little")


def digest(a: np.ndarray):
    b = np.ascontiguousarray(a, np.uint8).tobytes()
    return b.hex() if len(b) <= 64 else "sha256:" + hashlib.sha256(b).hexdigest()


def shards(tag, k, L):
    return [o.splitmix_bytes(seed_of(tag, k, L, j), L) for j in range(k)]


def field():
    return {
        "provenance": PROVENANCE,
        "polynomial": "0x11d",
        "generator": 2,
        "exp": o.exp_table().tobytes().hex(),
        "log": o.log_table().tobytes().hex(),
        "inv": bytes(o.gf_inv(a) for a in range(256)).hex(),
        "mul_samples": [[a, b, o.gf_mul(a, b)] for a, b in
                        [(2, 0x80), (0x53, 0xCA), (0xFF, 0xFF), (0, 7), (1, 0xAB), (0x8E, 2), (3, 7)]],
    }


def encode_cases():
    cases = []
    for k, m in CODES:
        enc = o.Encoder(k, m)
        mat = o.cauchy_matrix(k, m)
        for L in LENGTHS:
            if k * L > 10 * 65536 and L != 65536:
                continue
            data = shards("enc", k, L)
            par = enc.encode(data)
            cases.append({"k": k, "m": m, "L": L, "seeds": [seed_of("enc", k, L, j) for j in range(k)],
                          "parity": [digest(p) for p in par]})
    return {"provenance": PROVENANCE,
            "matrices": {f"{k},{m}": o.cauchy_matrix(k, m).tobytes().hex() for k, m in CODES},
            "tables": {f"{k},{m}": o.init_tables(o.cauchy_matrix(k, m)[k:]).tobytes().hex()
                       for k, m in [(4, 2), (8, 4)]},
            "cases": cases}


def decode_cases():
    out = []
    for (k, m), L in (((4, 2), 33), ((3, 2), 33), ((8, 4), 257)):
        data = shards("dec", k, L)
        par = o.Encoder(k, m).encode(data)
        units = data + par
        rng = np.random.default_rng(seed_of("order", k, m) & 0xFFFFFFFF)
        pats = [list(e) for n in range(1, m + 1) for e in itertools.combinations(range(k + m), n)]
        if len(pats) > 80:
            pats = [pats[i] for i in sorted(rng.choice(len(pats), 80, replace=False))]
        for erased in pats:
            for orderkind in ("sorted", "shuffled"):
                surv = [i for i in range(k + m) if i not in erased][:k]
                if orderkind == "shuffled":
                    surv = [int(x) for x in rng.permutation(surv)]
                for strict in (False, True):
                    rc, mat = o.decode_matrix(k, m, surv, erased, strict)
                    rc2, outs = o.decode(k, m, [units[i] for i in surv], surv, erased, strict)
                    out.append({"k": k, "m": m, "L": L, "decode_indexes": surv, "erased": erased,
                                "mode": "strict" if strict else "compat", "status": rc,
                                "matrix": mat.tobytes().hex(), "outputs": [digest(x) for x in outs]})
    # ELECT's own call shape (ECRecovery / ErasureCodeTest): decodeIndexes {4,1,2,3}, erase {0}
    k, m, L = 4, 2, 4099
    data = shards("elect", k, L)
    par = o.Encoder(k, m).encode(data)
    rc, outs = o.decode(k, m, [par[0], data[1], data[2], data[3]], [4, 1, 2, 3], [0])
    assert np.array_equal(outs[0], data[0])
    out.append({"k": k, "m": m, "L": L, "decode_indexes": [4, 1, 2, 3], "erased": [0], "mode": "compat",
                "status": rc, "matrix": o.decode_matrix(k, m, [4, 1, 2, 3], [0])[1].tobytes().hex(),
                "outputs": [digest(outs[0])], "input_seeds": [seed_of("elect", k, L, j) for j in range(k)]})
    # singular survivor set (duplicate index): compat keeps going like libec.so
    for strict in (False, True):
        rc, mat = o.decode_matrix(4, 2, [1, 1, 2, 3], [0], strict)
        out.append({"k": 4, "m": 2, "L": 0, "decode_indexes": [1, 1, 2, 3], "erased": [0],
                    "mode": "strict" if strict else "compat", "status": rc, "matrix": mat.tobytes().hex(),
                    "outputs": []})
    # singular survivor sets WITH bytes: libec.so ignores gf_invert_matrix's -1
    # (EC/erasure_coder.c:257-258) and codes with the partially reduced inverse
    # (:261-281), so the outputs are defined bytes, not an error; strict refuses.
    for (k, m), surv, erased in (((4, 2), [1, 1, 2, 3], [0]), ((4, 2), [4, 4, 5, 0], [1]),
                                 ((4, 2), [0, 1, 2, 2], [3, 4]), ((4, 2), [5, 4, 4, 1], [0, 2]),
                                 ((8, 4), [2, 2, 3, 4, 5, 6, 7, 8], [0, 1]),
                                 ((8, 4), [8, 9, 10, 11, 11, 0, 1, 2], [3, 4])):
        for L in (33, 4099):
            data = shards("sing", k, L)
            units = data + o.Encoder(k, m).encode(data)
            for strict in (False, True):
                rc, mat = o.decode_matrix(k, m, surv, erased, strict)
                assert rc == -1
                outs = [] if strict else o.decode(k, m, [units[i] for i in surv], surv, erased, False)[1]
                out.append({"k": k, "m": m, "L": L, "decode_indexes": surv, "erased": erased, "input_tag": "sing",
                            "mode": "strict" if strict else "compat", "status": rc, "singular": True,
                            "matrix": mat.tobytes().hex(), "outputs": [digest(x) for x in outs]})
    return {"provenance": PROVENANCE, "cases": out}


def update_cases():
    cases = []
    for k, m in ((4, 2), (8, 4)):
        enc = o.Encoder(k, m)
        for L in (1, 33, 4099):
            for t in range(k):
                old = o.splitmix_bytes(seed_of("upd-old", k, L, t), L)
                new = o.splitmix_bytes(seed_of("upd-new", k, L, t), L)
                pin = [o.splitmix_bytes(seed_of("upd-par", k, L, t, r), L) for r in range(m)]
                pout = enc.encode_update([old, new] + pin, t)
                cases.append({"k": k, "m": m, "L": L, "target": t, "parity_out": [digest(p) for p in pout]})
    return {"provenance": PROVENANCE, "seed_keys": "old: seed_of('upd-old',k,L,t); new: seed_of('upd-new',"
            "k,L,t); parity r: seed_of('upd-par',k,L,t,r)", "cases": cases}


def erasure_code_test_port(L=4099):
    """ErasureCodeTest.java:31-173 with codeLength = L instead of 419,483,300."""
    k, m = 4, 2
    rnd = JavaRandom(123)
    data = [rnd.nextBytes(L) for _ in range(k)]           # :58-67
    modified = [d.copy() for d in data]
    modified[0] = rnd.nextBytes(L)                         # :69-71
    enc = o.Encoder(k, m)
    parity = enc.encode(data)                              # :83
    second = enc.encode(modified)                          # :86
    _, out1 = o.decode(k, m, [parity[0]] + data[1:], [4, 1, 2, 3], [0])       # :107
    _, out2 = o.decode(k, m, [second[0]] + modified[1:], [4, 1, 2, 3], [0])   # :109
    upd = enc.encode_update([data[0], modified[0]] + parity, 0)              # :144
    return {
        "provenance": PROVENANCE + " Inputs: java.util.Random(123).nextBytes, JDK-specified LCG.",
        "codeLength": L,
        "data": [digest(d) for d in data],
        "modified0": digest(modified[0]),
        "parity": [digest(p) for p in parity],
        "second_parity": [digest(p) for p in second],
        "update_parity": [digest(p) for p in upd],
        "decode_original_equals_data0": bool(np.array_equal(out1[0], data[0])),
        "decode_updated_equals_modified0": bool(np.array_equal(out2[0], modified[0])),
        "update_equals_second_parity": all(np.array_equal(a, b) for a, b in zip(upd, second)),
        "head": {"data0": data[0][:16].tobytes().hex(), "parity0": parity[0][:16].tobytes().hex()},
    }


def main():
    files = {"gf_field.json": field(), "encode.json": encode_cases(), "decode.json": decode_cases(),
             "update.json": update_cases(), "erasure_code_test.json": erasure_code_test_port()}
    for name, obj in files.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
