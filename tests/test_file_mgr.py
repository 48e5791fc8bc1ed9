"""Native file-system client (BoxFileMgr / PaddleFileMgr contract,
box_wrapper.h:1016-1041; fs_open_read fw/io/fs.h:31-97).

Remote paths are exercised with a stand-in ``hadoop`` script that serves
``hdfs://cluster/...`` from a local directory and checks the ``-D`` options
the client passes, so the command lines the client builds are what is tested.
The pass loader reads a mixed filelist (local, local .gz, remote, remote .gz).
"""
import gzip
import os
import stat

import pytest

from paddlebox_amd import _native
from paddlebox_amd.utils.fs import BoxFileMgr, fs_open_read, fs_write

h = _native.host()

FAKE_HADOOP = r"""#!/bin/bash
# stand-in for `hadoop fs -D fs.default.name=X -D hadoop.job.ugi=Y -<verb> args`
ROOT="__ROOT__"
[ "$1" = fs ] || exit 9
shift
while [ "$1" = -D ]; do
  case "$2" in
    fs.default.name=hdfs://cluster) ;;
    hadoop.job.ugi=user,pass) ;;
    *) echo "bad option $2" >&2; exit 8 ;;
  esac
  shift 2
done
verb="$1"; shift
loc() { echo "$ROOT/${1#hdfs://cluster/}"; }
case "$verb" in
  -cat) cat "$(loc "$1")" ;;
  -text) zcat "$(loc "$1")" ;;
  -test) [ -e "$(loc "$2")" ] ;;
  -mkdir) mkdir -p "$(loc "$2")" ;;
  -rm) rm -rf "$(loc "$3")" ;;
  -mv) mv "$(loc "$1")" "$(loc "$2")" ;;
  -touchz) touch "$(loc "$1")" ;;
  -get) cp -r "$(loc "$1")" "$2" ;;
  -put) shift; if [ "$1" = - ]; then cat > "$(loc "$2")"; else cp -r "$1" "$(loc "$2")"; fi ;;
  -du) p="$(loc "$1")"; for f in "$p"/*; do echo "$(du -sb "$f" | cut -f1) hdfs://cluster/${f#$ROOT/}"; done ;;
  -ls) p="$(loc "$1")"
       if [ -d "$p" ]; then set -- "$p"/*; else set -- "$p"; fi
       for f in "$@"; do
         [ -e "$f" ] || exit 1
         t=-; [ -d "$f" ] && t=d
         echo "${t}rw-r--r--   3 user group $(stat -c %s "$f") 2026-01-01 00:00 hdfs://cluster/${f#$ROOT/}"
       done ;;
  *) exit 7 ;;
esac
"""


@pytest.fixture
def remote(tmp_path):
    root = tmp_path / "remote"
    root.mkdir()
    script = tmp_path / "hadoop"
    script.write_text(FAKE_HADOOP.replace("__ROOT__", str(root)))
    script.chmod(script.stat().st_mode | stat.S_IEXEC)
    fm = BoxFileMgr()
    assert fm.init("hdfs://cluster", "user,pass", hadoop_bin=str(script))
    yield fm, root
    fm.init("", "")  # back to local-only defaults for other tests


def test_local_ops(tmp_path):
    fm = BoxFileMgr()
    d = str(tmp_path / "a" / "b")
    assert fm.makedir(d) and fm.exists(d)
    assert fm.touch(d + "/x") and fm.file_size(d + "/x") == 0
    assert fs_write(d + "/y", b"hello world")
    assert fm.file_size(d + "/y") == 11
    assert fm.truncate(d + "/y", 5) and fs_open_read(d + "/y").read() == b"hello"
    assert fm.rename(d + "/y", d + "/z") and not fm.exists(d + "/y")
    assert fm.list_dir(d) == [d + "/x", d + "/z"]
    assert fm.count(d) == 2
    assert fm.dus(str(tmp_path / "a")) == [(d, 5)]
    assert fs_write(d + "/w.gz", b"zipped\n") and gzip.open(d + "/w.gz").read() == b"zipped\n"
    assert fs_open_read(d + "/w.gz").read() == b"zipped\n"
    assert fs_open_read(d + "/z", "tr a-z A-Z").read() == b"HELLO"
    assert fm.remove(d) and not fm.exists(d)


def test_remote_ops(remote, tmp_path):
    fm, root = remote
    base = "hdfs://cluster/data/day1"
    assert fm.makedir(base) and (root / "data/day1").is_dir()
    assert fm.exists(base) and not fm.exists(base + "/nope")
    assert fs_write(base + "/part-0", b"abc\n") and (root / "data/day1/part-0").read_bytes() == b"abc\n"
    assert fm.touch(base + "/donefile")
    assert fm.list_info(base) == [(base + "/donefile", 0), (base + "/part-0", 4)]
    assert fm.file_size(base + "/part-0") == 4 and fm.count(base) == 2
    assert fm.rename(base + "/part-0", base + "/part-1")
    assert fs_open_read(base + "/part-1").read() == b"abc\n"
    loc = str(tmp_path / "local" / "p1")
    assert fm.down(base + "/part-1", loc) and open(loc, "rb").read() == b"abc\n"
    assert fm.upload(loc, base + "/up") and (root / "data/day1/up").read_bytes() == b"abc\n"
    assert dict(fm.dus("hdfs://cluster/data"))["hdfs://cluster/data/day1"] > 0
    assert fm.remove(base + "/up") and not fm.exists(base + "/up")
    assert "-D fs.default.name='hdfs://cluster'" in fm._m.remote_prefix()


def test_loader_reads_remote_and_gz(remote, tmp_path):
    fm, root = remote
    lines = [f"1 {i % 2} 1 {100 + i}\n" for i in range(40)]
    (root / "d").mkdir()
    (root / "d" / "p0").write_text("".join(lines[0:10]))
    with gzip.open(root / "d" / "p1.gz", "wt") as f:
        f.write("".join(lines[10:20]))
    (tmp_path / "p2").write_text("".join(lines[20:30]))
    with gzip.open(tmp_path / "p3.gz", "wt") as f:
        f.write("".join(lines[30:40]))
    ds = h.SlotDataset()
    ds.set_slots([h.SlotDesc("label", "uint64", True, True, 1), h.SlotDesc("s", "uint64", True, False, 1)])
    ds.set_filelist(["hdfs://cluster/d/p0", "hdfs://cluster/d/p1.gz", str(tmp_path / "p2"), str(tmp_path / "p3.gz")])
    ds.set_thread_num(2)
    assert ds.load_into_memory() == 40
    assert sorted(ds.collect_keys(True).tolist()) == list(range(100, 140))
