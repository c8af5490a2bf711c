"""Philox4x32-10 counter RNG + Box-Muller normals + Feistel minibatch permutation (NumPy).

TEST INFRASTRUCTURE ONLY. Imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product path.

The reference draws noise with ``tf.random.normal`` (model/diffusion/diffusion_vpg.py:280,319)
and permutes minibatch rows with ``tf.random.shuffle``
(agent/finetune/train_ppo_diffusion_agent.py:287). TF's Philox streams cannot be reproduced
outside TF, so the MI355X build defines its OWN counter-based streams (documented in
DESIGN.md §RNG) and this file restates them bit-for-bit so that the in-kernel RNG path is
checkable too. Every integer here is exact; the normals differ from the device only by
fp32 transcendental rounding (checked with a tolerance in tests).
"""
import numpy as np

PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = np.uint64(0x9E3779B9)
PHILOX_W1 = np.uint64(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32 with 10 rounds. All inputs broadcastable uint32-valued arrays."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & _MASK32 for c in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint64) & _MASK32
    k1 = np.asarray(k1, dtype=np.uint64) & _MASK32
    for _ in range(10):
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _MASK32, lo1, (hi0 ^ c3 ^ k1) & _MASK32, lo0
        k0 = (k0 + PHILOX_W0) & _MASK32
        k1 = (k1 + PHILOX_W1) & _MASK32
    return c0, c1, c2, c3


def u32_to_unit(w):
    """(w >> 9 + 0.5) * 2^-23: exactly representable in fp32, strictly inside (0, 1)."""
    return ((np.asarray(w, dtype=np.uint64) >> np.uint64(9)).astype(np.float64) + 0.5) * (2.0 ** -23)


def box_muller4(w0, w1, w2, w3):
    """Four normals from one Philox block: pairs (w0,w1) and (w2,w3)."""
    u0, u1, u2, u3 = (u32_to_unit(w).astype(np.float32).astype(np.float64) for w in (w0, w1, w2, w3))
    r0 = np.sqrt(-2.0 * np.log(u0))
    r1 = np.sqrt(-2.0 * np.log(u2))
    a0 = 2.0 * np.pi * u1
    a1 = 2.0 * np.pi * u3
    return r0 * np.cos(a0), r0 * np.sin(a0), r1 * np.cos(a1), r1 * np.sin(a1)


def sampler_normals(seed, call_id, env_offset, n_env, n_elem, slot):
    """Normals used by the sampler for denoising slot ``slot`` (0..K-1 = loop index i,
    K = the initial x_T draw). Returns [n_env, n_elem] float64 (not yet clipped).

    counter = (elem // 4, global env row, slot, call_id); key = (seed lo, seed hi)."""
    seed = int(seed)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    n_grp = (n_elem + 3) // 4
    g = np.arange(n_grp, dtype=np.uint64)[None, :]
    e = (np.arange(n_env, dtype=np.uint64) + np.uint64(env_offset))[:, None]
    w = philox4x32_10(g, e, np.uint64(slot), np.uint64(call_id), k0, k1)
    z = np.stack(box_muller4(*w), axis=-1).reshape(n_env, n_grp * 4)
    return z[:, :n_elem]


def _feistel_round_keys(seed, epoch):
    seed = int(seed)
    w = philox4x32_10(np.uint64(epoch), np.uint64(0x5EED), np.uint64(0), np.uint64(0),
                      seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return [int(x) for x in w]


def _feistel(x, half_bits, keys):
    mask = (1 << half_bits) - 1
    x = np.asarray(x, dtype=np.uint64)
    left = (x >> np.uint64(half_bits)) & np.uint64(mask)
    right = x & np.uint64(mask)
    for k in keys:
        # round function: low bits of a multiply-xorshift hash of (right ^ key)
        h = (right ^ np.uint64(k)) & _MASK32
        h = (h * np.uint64(0x9E3779B1)) & _MASK32
        h = h ^ (h >> np.uint64(15))
        h = (h * np.uint64(0x85EBCA77)) & _MASK32
        h = h ^ (h >> np.uint64(13))
        left, right = right, (left ^ h) & np.uint64(mask)
    return (left << np.uint64(half_bits)) | right


def feistel_permute(i, n, seed, epoch):
    """Bijection of [0, n) used for PPO minibatch sampling (replaces tf.random.shuffle,
    train_ppo_diffusion_agent.py:287). 4-round balanced Feistel over [0, 4^h) >= n with
    cycle walking. Bit-identical to dppo_feistel_permute() in the HIP library."""
    n = int(n)
    half_bits = 1
    while (1 << (2 * half_bits)) < n:
        half_bits += 1
    keys = _feistel_round_keys(seed, epoch)
    x = np.asarray(i, dtype=np.uint64).copy()
    out = _feistel(x, half_bits, keys)
    bad = out >= np.uint64(n)
    while np.any(bad):
        out[bad] = _feistel(out[bad], half_bits, keys)
        bad = out >= np.uint64(n)
    return out.astype(np.int64)
