"""The seeded synthetic generator's doc-id shards (host code of the library, no GPU):
a shard of the collection quantized with the collection's max is exactly the global
collection's postings restricted to the shard's docs -- the multi-rank bench legs
build their shards this way (bench.retrieve_leg)."""
import numpy as np

from improving_learned_index_amd import synthetic as S


def test_shard_equals_the_global_collection_slice():
    n, v, seed = 12_000, 30_000, 11
    t_all, d_all, v_all, m_all = S.synth_postings(n, v, seed=seed)
    cuts = [0, 5_000, 9_000, n]
    maxima = [S.synth_max_impact(b - a, v, seed=seed, doc0=a) for a, b in zip(cuts, cuts[1:])]
    assert max(maxima) == m_all
    for a, b in zip(cuts, cuts[1:]):
        t_s, d_s, v_s, m_s = S.synth_postings(b - a, v, seed=seed, doc0=a, quant_max=m_all)
        assert m_s == S.synth_max_impact(b - a, v, seed=seed, doc0=a)
        for t in range(0, v, 97):
            g = slice(t_all[t], t_all[t + 1])
            keep = (d_all[g] >= a) & (d_all[g] < b)
            want = list(zip((d_all[g][keep] - a).tolist(), v_all[g][keep].tolist()))
            got = list(zip(d_s[t_s[t]:t_s[t + 1]].tolist(), v_s[t_s[t]:t_s[t + 1]].tolist()))
            assert got == want, (a, t)


def test_quantize_like_reference_takes_the_collection_max():
    imp = np.array([0.5, 1.25, 2.0], np.float32)
    q, m = S.quantize_like_reference(imp, max_val=4.0)
    assert m == 4.0 and q.tolist() == [31, 79, 127]
