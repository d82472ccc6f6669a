"""CPU: pin the oracle to the reference's own golden vectors and check its
internal consistency (ref_layout vs compact vs lean).  No GPU."""
import json
import os
import random

import numpy as np
import pytest

from conftest import CONFIG_SCORES, FASTA, GOLDEN, TEST_SCORES, read_fasta_records


def _ref_cases():
    with open(os.path.join(GOLDEN, "reference_vectors.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", _ref_cases()["cases"], ids=lambda c: c["name"])
@pytest.mark.parametrize("layout", [0, 1], ids=["compact", "ref_layout"])
def test_oracle_reference_golden(oracle, case, layout):
    r = oracle.align(case["s1"].encode(), case["s2"].encode(), tuple(_ref_cases()["scores"]),
                     is_local=case["is_local"], layout=layout)
    assert r.status == 0
    if case["score"] is not None:
        assert r.score == case["score"]
    assert r.matches == case["matches"]
    assert r.mismatches == case["mismatches"]
    assert r.opening_gaps == case["opening_gaps"]
    assert r.gap_extensions == case["gap_extensions"]
    assert [list(x) for x in r.alignment()] == case["alignment"]


def test_oracle_committed_vectors(oracle):
    """Committed golden fixtures (tests/golden/oracle_vectors.json, made by
    tests/golden/make_golden.py) still reproduce."""
    with open(os.path.join(GOLDEN, "oracle_vectors.json")) as f:
        data = json.load(f)
    for c in data["cases"]:
        r = oracle.align(c["s1"].encode("latin-1"), c["s2"].encode("latin-1"), tuple(c["scores"]),
                         is_local=c["is_local"])
        assert r.score == c["score"], c["name"]
        assert [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps] == c["stats"], c["name"]
        assert list(r.start) == c["start"] and list(r.max_cell) == c["max_cell"], c["name"]
        assert r.matches_at_max == c["matches_at_max"], c["name"]
        assert [list(x) for x in r.alignment()] == c["alignment"], c["name"]


def test_survey_appendix_b_config1(oracle):
    """BANANA x MISSISSIPPI under config.toml."""
    g = oracle.align(b"BANANA", b"MISSISSIPPI", CONFIG_SCORES, is_local=False)
    assert (g.score, len(g.choices), g.start, g.matches, g.mismatches, g.opening_gaps, g.gap_extensions,
            g.max_cell, g.matches_at_max) == (-22, 11, (6, 11), 1, 5, 1, 4, (1, 1), 0)
    assert g.alignment()[0] == ("Match", 6, 11)       # None == None quirk
    loc = oracle.align(b"BANANA", b"MISSISSIPPI", CONFIG_SCORES, is_local=True)
    assert (loc.score, len(loc.choices), loc.start) == (0, 11, (6, 11))
    assert all(c == "Insert" or c == "OpenInsert" for c, _, _ in loc.alignment())


def test_layouts_agree_random(oracle):
    rng = random.Random(7)
    for _ in range(60):
        n, m = rng.randint(0, 30), rng.randint(0, 30)
        a = bytes(rng.choice(b"ACGT") for _ in range(n))
        b = bytes(rng.choice(b"ACGT") for _ in range(m))
        for loc in (False, True):
            r0 = oracle.align(a, b, CONFIG_SCORES, is_local=loc, layout=0, want_planes=True)
            r1 = oracle.align(a, b, CONFIG_SCORES, is_local=loc, layout=1, want_planes=True)
            rl = oracle.align_lean(a, b, CONFIG_SCORES, is_local=loc)
            assert r0.alignment() == r1.alignment() == rl.alignment()
            assert np.array_equal(r0.planes, r1.planes)
            assert (r0.score, r0.start, r0.max_cell, r0.matches_at_max) == \
                   (rl.score, rl.start, rl.max_cell, rl.matches_at_max)


def test_local_tracebacks_end_on_boundary(oracle):
    """local walks never stop in the interior."""
    rng = random.Random(3)
    for _ in range(100):
        a = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(1, 25)))
        b = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(1, 25)))
        r = oracle.align(a, b, CONFIG_SCORES, is_local=True)
        if len(r.choices):
            c, i, j = r.alignment()[-1]
            # the last pushed step moves onto row 0 or column 0 (or stops there)
            assert i <= 1 or j <= 1


def test_oracle_fasta_parse(oracle):
    recs = read_fasta_records(os.path.join(FASTA, "test3_short.fasta"))
    assert recs == [(b"s1", b"GCATGCG"), (b"s2", b"GATTACA")]
    recs = read_fasta_records(os.path.join(FASTA, "Human-Mouse-BRCA2-cds.fasta"))
    assert len(recs) == 2 and len(recs[0][1]) == 11382 and len(recs[1][1]) == 10346


def test_oracle_fasta_edge_cases(oracle):
    data = b"junk before header\n>  name one \r\nAC GT \n\n  \n>two\n\tAAA\t\n>empty\n"
    assert oracle.fasta_parse(data) == [(b"name one", b"AC GT"), (b"two", b"AAA"), (b"empty", b"")]
    # reading stops at the first invalid UTF-8 line (map_while(Result::ok))
    assert oracle.fasta_parse(b">a\nAC\n\xff\xfe\nGG\n") == [(b"a", b"AC")]
