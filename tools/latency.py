#!/usr/bin/env python3
"""Per-record latency of the trait-object path (Encryptor::encrypt /
Decryptor::decrypt -> sg_seal / sg_open, one record per call, host memory in
and out): the path TlsWriter::write_record takes when records are not
batched.  Prints one JSON line per record size."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from suruga_amd import ChaCha20Poly1305  # noqa: E402


def main():
    aead = ChaCha20Poly1305(0)
    enc, dec = aead.new_encryptor(bytes(range(32))), aead.new_decryptor(bytes(range(32)))
    ad = bytes(13)
    for n in (16, 1024, 16384):
        pt = bytes(n)
        nonce = bytes(8)
        for _ in range(20):
            ct = enc.encrypt(nonce, pt, ad)
        reps = 500
        t0 = time.perf_counter()
        for i in range(reps):
            ct = enc.encrypt(nonce, pt, ad)
        t1 = time.perf_counter()
        for i in range(reps):
            dec.decrypt(nonce, ct, ad)
        t2 = time.perf_counter()
        print(json.dumps({"record_bytes": n, "seal_us": round((t1 - t0) / reps * 1e6, 1),
                          "open_us": round((t2 - t1) / reps * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
