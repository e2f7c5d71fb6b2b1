"""Fixture key helpers shared by tests (tests/golden/make_golden.py:107 naming)."""


def trad_key(algo, alpha, es):
    return f"ms_a{alpha}_es{int(es)}" if algo == "ms" else f"bp_es{int(es)}"
