"""GPU: the chunked build's growing key set (g2n_keyset_*, HipEngine.keyset): ids in insertion
order across calls (builders.py:194-198 first-touch minting over chunks), keys of any length
(empty included), growth past the first table, and the set's names in id order — against a Python
dict.  The chunked general build itself is covered by tests/test_gpu_shard.py."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _batch(r, pool, n):
    keys = list(dict.fromkeys(r.choice(pool) for _ in range(n)))  # distinct within one call
    offs = np.zeros(len(keys) + 1, dtype=np.int64)
    np.cumsum([len(k) for k in keys], out=offs[1:])
    return keys, np.frombuffer(b"".join(keys), dtype=np.uint8).copy(), offs


def test_keyset_matches_dict(gpu):
    import torch

    from gfa2network_amd.shard import HipEngine

    r = random.Random(4)
    pool = [b""] + [bytes(r.choice(b"ACGTacgt_:+-0123456789") for _ in range(r.choice([1, 3, 8, 16, 17, 40, 200])))
                    for _ in range(60000)]
    pool = list(dict.fromkeys(pool))
    eng = HipEngine(0)
    ks = eng.keyset()
    ref = {}
    try:
        for step in range(7):
            keys, blob, offs = _batch(r, pool, [10, 5000, 20000, 1, 0, 30000, 8000][step])
            ids, n_tot = ks.add(torch.from_numpy(blob).to(eng.device), torch.from_numpy(offs).to(eng.device))
            want = []
            for k in keys:
                ref.setdefault(k, len(ref))
                want.append(ref[k])
            assert ids.cpu().numpy().tolist() == want, step
            assert n_tot == len(ref), step
        nb, no = ks.names()
        nb, no = nb.cpu().numpy().tobytes(), no.cpu().numpy()
        got = [nb[no[i]:no[i + 1]] for i in range(len(no) - 1)]
        assert got == list(ref), "names in id order"
    finally:
        ks.close()
        eng.close()


def test_keyset_refuses_keys_past_its_length_field(gpu):
    """A key of 2^24 bytes or more does not fit KsEntry's 24-bit length: the add is refused
    (G2N_E_UNSUPPORTED) instead of storing a truncated length that later lookups would miss
    (ADVICE r05); one byte shorter is accepted and found again."""
    import torch

    from gfa2network_amd.shard import HipEngine

    eng = HipEngine(0)
    ks = eng.keyset()
    try:
        for n, ok in ((1 << 24) - 1, True), (1 << 24, False):
            key = np.full(n, ord("a"), dtype=np.uint8)
            key[-1] = ord("z") if ok else ord("y")
            offs = np.array([0, 1, 1 + n], dtype=np.int64)
            blob = np.concatenate([np.array([ord("k")], dtype=np.uint8), key])
            args = (torch.from_numpy(blob).to(eng.device), torch.from_numpy(offs).to(eng.device))
            if ok:
                ids, n_tot = ks.add(*args)
                assert ids.cpu().numpy().tolist() == [0, 1] and n_tot == 2
                ids, n_tot = ks.add(*args)  # found again, nothing new
                assert ids.cpu().numpy().tolist() == [0, 1] and n_tot == 2
            else:
                with pytest.raises(RuntimeError, match="UNSUPPORTED"):
                    ks.add(*args)
    finally:
        ks.close()
        eng.close()
