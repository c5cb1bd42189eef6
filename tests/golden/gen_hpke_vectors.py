"""Extracts the RFC 9180 test vectors of the HPKE suites the GPU opener implements
(mode_base, DHKEM(X25519, HKDF-SHA256) 0x0020 or DHKEM(P-256, HKDF-SHA256) 0x0010, HKDF-SHA256
0x0001, with AES-128-GCM 0x0001, AES-256-GCM 0x0002 and ChaCha20Poly1305 0x0003) from the
file Janus's own HPKE test reads (/root/reference/core/src/test-vectors.json, used by
core/src/hpke.rs `decrypt_test_vectors`).  Run in the build container only; the output fixture is
data (keys, ciphertexts, plaintexts), committed as tests/golden/hpke_rfc9180_x25519.json."""
import json
import os
import sys

SRC = "/root/reference/core/src/test-vectors.json"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hpke_rfc9180_x25519.json")


# (aead id, output file): AES-128-GCM (the original fixture), AES-256-GCM, ChaCha20Poly1305
_D = os.path.dirname(OUT)
OUTS = {(32, 1): OUT,
        (32, 2): os.path.join(_D, "hpke_rfc9180_x25519_aes256gcm.json"),
        (32, 3): os.path.join(_D, "hpke_rfc9180_x25519_chacha20poly1305.json"),
        (16, 1): os.path.join(_D, "hpke_rfc9180_p256_aes128gcm.json"),
        (16, 2): os.path.join(_D, "hpke_rfc9180_p256_aes256gcm.json"),
        (16, 3): os.path.join(_D, "hpke_rfc9180_p256_chacha20poly1305.json")}
ALL_OUT = os.path.join(_D, "hpke_rfc9180_all.json")


def main():
    vecs = json.load(open(SRC))
    for (kem, aead), path in OUTS.items():
        keep = [v for v in vecs
                if (v["mode"], v["kem_id"], v["kdf_id"], v["aead_id"]) == (0, kem, 1, aead)]
        if len(keep) != 1:
            sys.exit(f"expected exactly one kem {kem} / HKDF-SHA256 / aead {aead} base-mode vector")
        v = keep[0]
        out = {k: v[k] for k in ("mode", "kem_id", "kdf_id", "aead_id", "info", "enc", "pkRm",
                                 "skRm", "base_nonce")}
        out["encryptions"] = v["encryptions"][:4]
        out["source"] = ("RFC 9180 test-vector set, core/src/test-vectors.json (read by Janus's "
                         "hpke.rs decrypt_test_vectors)")
        json.dump(out, open(path, "w"), indent=1)
        print("wrote", path)
    # every base-mode vector of the file: 4 KEMs (X25519, P-256, X448, P-521)
    # x 2 KDFs (HKDF-SHA256, HKDF-SHA512) x 3 AEADs = 24, each with its base_nonce encryption
    allv = []
    for v in vecs:
        if v["mode"] != 0:
            continue
        e = [x for x in v["encryptions"] if x["nonce"] == v["base_nonce"]]
        out = {k: v[k] for k in ("mode", "kem_id", "kdf_id", "aead_id", "info", "enc", "pkRm",
                                 "skRm", "base_nonce")}
        out["encryptions"] = e[:1]
        allv.append(out)
    if len(allv) != 24:
        sys.exit(f"expected 24 base-mode vectors, found {len(allv)}")
    json.dump({"source": "RFC 9180 test-vector set, core/src/test-vectors.json (read by Janus's "
                         "hpke.rs decrypt_test_vectors)", "vectors": allv},
              open(ALL_OUT, "w"), indent=1)
    print("wrote", ALL_OUT)


if __name__ == "__main__":
    main()
