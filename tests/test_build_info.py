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


def test_no_hip_object_older_than_its_headers():
    """Every HIP object of the in-tree build is newer than every header: torch's
    ninja build gives hipcc no depfile, so a header change (a struct field
    added to kernels.h) used to leave .hip objects compiled with the old
    layout -- kernel arguments at shifted offsets, a GPU memory fault
    (setup.py now drops such objects before building)."""
    import glob
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    objs = glob.glob(os.path.join(root, "build", "temp.*", "csrc", "hip", "*.o"))
    if not objs:
        pytest.skip("no in-tree build directory")
    headers = glob.glob(os.path.join(root, "csrc", "hip", "*.h")) + glob.glob(os.path.join(root, "csrc", "common", "*.h"))
    newest = max(os.path.getmtime(h) for h in headers)
    stale = [os.path.basename(o) for o in objs if os.path.getmtime(o) < newest]
    assert not stale, f"HIP objects older than the newest header: {stale} (run __graft_entry__.build())"
