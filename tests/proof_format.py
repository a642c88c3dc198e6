"""Section parser of the proof wire format zkp_prove / the oracle write
(winterfell 0.12 `Proof::to_bytes` as restated in SURVEY.md Appendix A and
DESIGN.md §2). Test helper: splits a proof into its byte sections so stage
outputs can be compared with the matching part of a whole proof."""


class Reader:
    def __init__(self, b: bytes):
        self.b, self.o = b, 0

    def take(self, k: int) -> bytes:
        v = self.b[self.o:self.o + k]
        assert len(v) == k, "truncated proof"
        self.o += k
        return v

    def uint(self, k: int) -> int:
        return int.from_bytes(self.take(k), "little")


def sections(proof: bytes) -> dict:
    """-> {context, num_queries, commitments, queries (u8 1 + trace/constraint openings),
    ood_trace, ood_comp, fri_queries (u8 L + layers), remainder, nonce}: raw bytes per part."""
    r = Reader(proof)
    out = {}
    start = r.o
    r.take(6)                      # trace info: width, aux, aux rands, log2 n, meta len
    r.take(1 + 16)                 # modulus byte length + modulus
    r.take(8)                      # options
    r.take(4)                      # num constraints
    out["context"] = proof[start:r.o]
    out["num_queries"] = r.uint(1)
    out["commitments"] = r.take(r.uint(2))
    q0 = r.o
    assert r.uint(1) == 1          # one trace segment
    for _ in range(2):             # trace, constraint: values, batch paths
        r.take(r.uint(4))
        r.take(r.uint(4))
    out["queries"] = proof[q0:r.o]
    ood_len = r.uint(2)
    ood = r.take(ood_len)
    out["ood_trace"] = ood[1:]     # u8(2) then [T(z) | T(zg)] row by row
    out["ood_comp"] = r.take(r.uint(2))
    f0 = r.o
    nl = r.uint(1)
    for _ in range(nl):
        r.take(r.uint(4))
        r.take(r.uint(4))
    out["fri_queries"] = proof[f0:r.o]
    out["remainder"] = r.take(r.uint(2))
    assert r.uint(1) == 1          # num partitions
    out["nonce"] = r.uint(8)
    assert r.uint(1) == 0          # no GKR proof
    assert r.o == len(proof)
    return out
