"""Build provenance: the in-tree libraries carry a stamp of the sources they
were built from (__graft_entry__.build), and it matches this tree."""
import pytest

from paddlebox_amd import _native


def test_sources_digest_is_stable():
    assert _native.sources_digest() == _native.sources_digest()
    assert len(_native.sources_digest()) == 16


def test_build_stamp_matches_tree():
    info = _native.build_info()
    if info["stamp"] is None:
        pytest.skip("no build stamp (extensions built without __graft_entry__.build)")
    assert info["stamp"]["arch"] == "gfx950"
    assert info["matches_tree"], f"in-tree libraries are stale: built from {info['stamp']['sources']}, " \
                                 f"tree is {info['sources_now']} (rebuild with __graft_entry__.build())"
