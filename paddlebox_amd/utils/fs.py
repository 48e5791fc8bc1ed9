"""File-system client: ``BoxFileMgr`` (reference ``box_helper_py.cc:167-216``,
``box_wrapper.h:1016-1041``, ``box_wrapper.cc:1326-1397``) over the native
``FileMgr`` (``csrc/host/file_mgr.{h,cc}``).

Local paths are served with POSIX calls; ``hdfs://`` / ``afs://`` paths go
through the cluster's ``hadoop fs`` command line configured by ``init``
(``fs_name`` -> ``-D fs.default.name``, ``fs_ugi`` -> ``-D hadoop.job.ugi``,
``conf_path`` -> ``--config``), like Paddle's ``fw/io/fs.h`` hdfs functions.
The pass loaders open every data file through the same native client, so
``BoxFileMgr.init`` also makes remote and ``.gz`` filelists loadable.
"""
from __future__ import annotations

import io
from typing import List, Tuple

from .. import _native


class BoxFileMgr:
    def __init__(self):
        self._m = _native.host().default_file_mgr()
        self.inited = False

    def init(self, fs_name: str = "", fs_ugi: str = "", conf_path: str = "", expire_time: int = 0,
             hadoop_bin: str = "") -> bool:
        self.inited = bool(self._m.init(fs_name, fs_ugi, conf_path, hadoop_bin))
        return self.inited

    def list_dir(self, path: str) -> List[str]:
        return self._m.list_dir(path)

    def makedir(self, path: str) -> bool:
        return self._m.makedir(path)

    def exists(self, path: str) -> bool:
        return self._m.exists(path)

    def down(self, remote: str, local: str) -> bool:
        return self._m.download(remote, local)

    download = down

    def upload(self, local: str, remote: str) -> bool:
        return self._m.upload(local, remote)

    def remove(self, path: str) -> bool:
        return self._m.remove(path)

    def file_size(self, path: str) -> int:
        return self._m.file_size(path)

    def dus(self, path: str) -> List[Tuple[str, int]]:
        """(entry, bytes incl. subtree) for each entry of ``path``."""
        return self._m.dus(path)

    def truncate(self, path: str, size: int) -> bool:
        return self._m.truncate(path, int(size))

    def touch(self, path: str) -> bool:
        return self._m.touch(path)

    def rename(self, src: str, dst: str) -> bool:
        return self._m.rename(src, dst)

    def list_info(self, path: str) -> List[Tuple[str, int]]:
        return self._m.list_info(path)

    def count(self, path: str) -> int:
        return self._m.count(path)

    def destory(self):  # the reference's spelling
        self._m.destroy()
        self.inited = False

    finalize = destory


def fs_open_read(path: str, pipe_command: str = "cat") -> io.BytesIO:
    """Whole-file read through the loaders' open path (``fs_open_read``:
    local / remote, plain / .gz, optional converter command)."""
    return io.BytesIO(_native.host().default_file_mgr().read_bytes(path, pipe_command or ""))


def fs_write(path: str, data: bytes) -> bool:
    """Write a whole file (local, .gz, or remote via ``hadoop fs -put -``)."""
    return _native.host().default_file_mgr().write_bytes(path, data)
