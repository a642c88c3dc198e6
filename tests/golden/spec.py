"""Pure-Python restatements used ONLY to generate / cross-check golden fixtures.

TEST INFRASTRUCTURE — never imported by the product path.

* f128: winter-math `f128::BaseElement` (winterfell 0.12, crate not vendored —
  SURVEY.md F1/F3): p = 2^128 - 45*2^40 + 1, GENERATOR = 3, TWO_ADICITY = 40.
* BLAKE3: the published BLAKE3 specification (blake3 crate 1.5.4 is the
  reference's pinned dependency, Cargo.lock:195-205); pinned here by the
  published digests of "" and "abc" (SURVEY.md Appendix D).
* MiMC / f64_to_felt / get_round_constants: /root/reference/src/helper.rs:25-27,
  213-233, 404-406.
"""

P = 2**128 - 45 * 2**40 + 1
G = 3
TWO_ADICITY = 40
TWO_ADIC_ROOT = pow(G, (P - 1) >> TWO_ADICITY, P)
MASK128 = (1 << 128) - 1


def felt_new(v: int) -> int:
    """`BaseElement::new(u128)`: one conditional subtraction (2p > 2^128)."""
    v &= MASK128
    return v - P if v >= P else v


def root_of_unity(log_n: int) -> int:
    """`StarkField::get_root_of_unity(n)` = ROOT^(2^(40-n))."""
    return pow(TWO_ADIC_ROOT, 1 << (TWO_ADICITY - log_n), P)


def inv(a: int) -> int:
    return 0 if a == 0 else pow(a, P - 2, P)


# ---------------------------------------------------------------- helper.rs
def f64_to_felt(x: float) -> int:
    """helper.rs:25-27 — `Felt::new((x * 1e6).round() as u128)`.

    Rust `f64::round` is half-away-from-zero and `as u128` saturates
    (negatives and NaN -> 0, overflow -> u128::MAX)."""
    import math

    y = x * 1e6
    if y != y:  # NaN
        return 0
    r = math.floor(abs(y) + 0.5)
    r = -r if y < 0 else r
    if r <= 0:
        return 0
    if r >= 2**128:
        r = 2**128 - 1
    return felt_new(int(r))


def get_round_constants():
    """helper.rs:404-406 — (1..=64).map(|i| f64_to_felt(i))."""
    return [f64_to_felt(float(i)) for i in range(1, 65)]


def mimc_cipher(x: int, rc: int, z: int) -> int:
    """helper.rs:213-220."""
    for _ in range(64):
        x = pow((x + rc + z) % P, 7, P)
    return (x + z) % P


def mimc_hash_matrix(w, b, rcs) -> int:
    """helper.rs:222-233."""
    z = 0
    for i in range(len(w)):
        for j in range(len(w[i])):
            z = mimc_cipher(w[i][j], rcs[j % len(rcs)], z)
        z = mimc_cipher(b[i], rcs[i % len(rcs)], z)
    return z


# ---------------------------------------------------------------- BLAKE3
_IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
       0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
_PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
CHUNK_START, CHUNK_END, PARENT, ROOT = 1, 2, 4, 8
_M32 = 0xFFFFFFFF


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & _M32


def _g(s, a, b, c, d, mx, my):
    s[a] = (s[a] + s[b] + mx) & _M32
    s[d] = _rotr(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & _M32
    s[b] = _rotr(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b] + my) & _M32
    s[d] = _rotr(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & _M32
    s[b] = _rotr(s[b] ^ s[c], 7)


def compress(cv, block: bytes, counter: int, block_len: int, flags: int):
    block = block + b"\0" * (64 - len(block))
    m = [int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)]
    s = list(cv) + _IV[:4] + [counter & _M32, (counter >> 32) & _M32, block_len, flags]
    for r in range(7):
        _g(s, 0, 4, 8, 12, m[0], m[1]); _g(s, 1, 5, 9, 13, m[2], m[3])
        _g(s, 2, 6, 10, 14, m[4], m[5]); _g(s, 3, 7, 11, 15, m[6], m[7])
        _g(s, 0, 5, 10, 15, m[8], m[9]); _g(s, 1, 6, 11, 12, m[10], m[11])
        _g(s, 2, 7, 8, 13, m[12], m[13]); _g(s, 3, 4, 9, 14, m[14], m[15])
        if r < 6:
            m = [m[_PERM[i]] for i in range(16)]
    return [s[i] ^ s[i + 8] for i in range(8)]


def _chunk_cv(chunk: bytes, idx: int, root: bool):
    cv = list(_IV)
    blocks = [chunk[i:i + 64] for i in range(0, len(chunk), 64)] or [b""]
    for bi, blk in enumerate(blocks):
        fl = (CHUNK_START if bi == 0 else 0) | (CHUNK_END if bi == len(blocks) - 1 else 0)
        if root and bi == len(blocks) - 1:
            fl |= ROOT
        cv = compress(cv, blk, idx, len(blk), fl)
    return cv


def _subtree(chunks, first, root):
    if len(chunks) == 1:
        return _chunk_cv(chunks[0], first, root)
    left = 1 << ((len(chunks) - 1).bit_length() - 1)
    l = _subtree(chunks[:left], first, False)
    r = _subtree(chunks[left:], first + left, False)
    words = b"".join(x.to_bytes(4, "little") for x in l + r)
    return compress(list(_IV), words, 0, 64, PARENT | (ROOT if root else 0))


def blake3(data: bytes) -> bytes:
    chunks = [data[i:i + 1024] for i in range(0, len(data), 1024)] or [b""]
    out = _subtree(chunks, 0, True)
    return b"".join(x.to_bytes(4, "little") for x in out)


def felts_to_bytes(vals) -> bytes:
    return b"".join(int(v).to_bytes(16, "little") for v in vals)


def hash_elements(vals) -> bytes:
    """winter-crypto `Blake3_256::hash_elements` for f128 (IS_CANONICAL)."""
    return blake3(felts_to_bytes(vals))


def merge(a: bytes, b: bytes) -> bytes:
    return blake3(a + b)


def merge_with_int(seed: bytes, v: int) -> bytes:
    return blake3(seed + int(v).to_bytes(8, "little"))


# ---------------------------------------------------------------- NTT (naive)
def eval_poly(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % P
    return acc


def naive_lde(values, blowup, offset=G):
    """Interpolate `values` over <w_n> then evaluate on offset*<w_{n*blowup}>."""
    n = len(values)
    w = root_of_unity(n.bit_length() - 1)
    winv = inv(w)
    ninv = inv(n)
    coeffs = [sum(values[j] * pow(winv, j * k, P) for j in range(n)) * ninv % P for k in range(n)]
    N = n * blowup
    wN = root_of_unity(N.bit_length() - 1)
    return coeffs, [eval_poly(coeffs, offset * pow(wN, i, P) % P) for i in range(N)]


def merkle_root(leaves):
    """winter-crypto MerkleTree::new: nodes[i] = merge(nodes[2i], nodes[2i+1])."""
    level = list(leaves)
    while len(level) > 1:
        level = [merge(level[2 * i], level[2 * i + 1]) for i in range(len(level) // 2)]
    return level[0]


# ---------------------------------------------------------------- ChaCha (rand 0.8 StdRng)
# StdRng = rand_chacha ChaCha12Rng (rand 0.8, Cargo.lock): state = "expand 32-byte k",
# key = the 32-byte seed, 64-bit block counter in words 12-13 (from 0), 64-bit stream
# id 0 in words 14-15; output block = rounds(state) + state, 16 LE u32 words;
# RngCore::next_u64 reads words (2i, 2i+1) as lo | hi << 32 (rand_core BlockRng).
def _chacha_block(key: bytes, counter: int, nonce_words, rounds: int):
    M = 0xFFFFFFFF
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    s += [int.from_bytes(key[4 * i:4 * i + 4], "little") for i in range(8)]
    s += [counter & M] + list(nonce_words)
    x = list(s)

    def rotl(v, n):
        return ((v << n) | (v >> (32 - n))) & M

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & M; x[d] = rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & M; x[b] = rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & M; x[d] = rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & M; x[b] = rotl(x[b] ^ x[c], 7)
    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(a + b) & M for a, b in zip(x, s)]


def chacha20_block_rfc8439(key: bytes, counter: int, nonce: bytes):
    """RFC 8439 §2.3 layout (32-bit counter, 96-bit nonce): the published test vector pins the core."""
    return _chacha_block(key, counter, [int.from_bytes(nonce[4 * i:4 * i + 4], "little") for i in range(3)], 20)


def stdrng_next_u64(seed: bytes, count: int):
    """First `count` next_u64() of rand 0.8 `StdRng::from_seed(seed)` (ChaCha12, counter 0, stream 0)."""
    words = []
    blk = 0
    while len(words) < 2 * count:
        words += _chacha_block(seed, blk, [0, 0, 0], 12)  # block counter < 2^32 here: high word 0
        blk += 1
    return [words[2 * i] | (words[2 * i + 1] << 32) for i in range(count)]
