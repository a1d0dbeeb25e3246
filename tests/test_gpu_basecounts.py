"""Per-segment base counts (transform_state_t.base_count_unique /
base_count_nonunique, hpp:61-62 -- declared and zeroed by the reference, never
computed) on the GPU against the oracle restatement (oracle_base_counts), through
every route that builds an archive: one call, virtual shards, streamed
ingestion.  With the option off, the archive is unchanged byte for byte."""
import json

import pytest

from tests import corpus, oracle_lib

pytestmark = pytest.mark.gpu


def _ctx(bc=True):
    import starch_amd
    c = starch_amd.Starch(0)
    c.base_counts = bc
    return c


def _inputs():
    import starch_amd
    yield "hg38", starch_amd.gen_bed(0, 300_000)
    yield "narrowPeak", starch_amd.gen_bed(1, 60_000)
    for seed in range(3):
        yield "quirky%d" % seed, (corpus.fuzz_bed(seed, 2000) + corpus.multi_chrom_bed(4, 300, seed, "bed6") +
                                  corpus.parseable_fuzz_bed(seed, 1500) + b"chr9\tx\ty\nchr9\t1")
    yield "overlaps", b"".join(b"chrO\t%d\t%d\n" % (i * 7, i * 7 + (i % 23) * 3 + 1) for i in range(50_000))
    yield "empty", b""


@pytest.mark.parametrize("name,data", list(_inputs()), ids=lambda x: x if isinstance(x, str) else "")
def test_base_counts_match_oracle(name, data):
    import starch_amd
    want = oracle_lib.base_counts(data)
    c = _ctx()
    arch = c.compress(data)
    got = [(s.base_count_unique, s.base_count_nonunique) for _, s in c.segments()]
    assert got == want
    idx, streams = starch_amd.parse_archive(arch)
    assert [(m["uniqueBaseCount"], m["nonUniqueBaseCount"]) for m in idx["streams"]] == want
    c.close()
    # the streams are the same with the option off; only the index differs
    c0 = _ctx(False)
    arch0 = c0.compress(data)
    idx0, streams0 = starch_amd.parse_archive(arch0)
    assert streams0 == streams
    assert all("uniqueBaseCount" not in m for m in idx0["streams"])
    c0.close()


def test_base_counts_sharded_and_streamed():
    import starch_amd
    data = starch_amd.gen_bed(0, 200_000) + corpus.fuzz_bed(5, 800)
    ref = _ctx()
    one = ref.compress(data)
    ref.close()
    ctxs = [_ctx() for _ in range(3)]
    assert starch_amd.compress_multi(ctxs, data) == one
    for c in ctxs:
        c.close()
    c = _ctx()
    assert c.compress_stream([data[i:i + 100_003] for i in range(0, len(data), 100_003)], batch_bytes=1) == one
    c.close()
    idx, _ = starch_amd.parse_archive(one)
    assert [(m["uniqueBaseCount"], m["nonUniqueBaseCount"]) for m in idx["streams"]] == oracle_lib.base_counts(data)
