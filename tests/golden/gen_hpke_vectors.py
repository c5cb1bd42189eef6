"""Extracts the RFC 9180 test vector(s) of the HPKE suite the GPU opener implements
(mode_base, DHKEM(X25519, HKDF-SHA256) 0x0020, HKDF-SHA256 0x0001, AES-128-GCM 0x0001) from the
file Janus's own HPKE test reads (/root/reference/core/src/test-vectors.json, used by
core/src/hpke.rs `decrypt_test_vectors`).  Run in the build container only; the output fixture is
data (keys, ciphertexts, plaintexts), committed as tests/golden/hpke_rfc9180_x25519.json."""
import json
import os
import sys

SRC = "/root/reference/core/src/test-vectors.json"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hpke_rfc9180_x25519.json")


def main():
    vecs = json.load(open(SRC))
    keep = [v for v in vecs if (v["mode"], v["kem_id"], v["kdf_id"], v["aead_id"]) == (0, 32, 1, 1)]
    if len(keep) != 1:
        sys.exit("expected exactly one X25519/HKDF-SHA256/AES-128-GCM base-mode vector")
    v = keep[0]
    out = {k: v[k] for k in ("mode", "kem_id", "kdf_id", "aead_id", "info", "enc", "pkRm", "skRm",
                             "base_nonce")}
    out["encryptions"] = v["encryptions"][:4]
    out["source"] = "RFC 9180 Appendix A.1.1 via core/src/test-vectors.json"
    json.dump(out, open(OUT, "w"), indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
