"""File-system client (BoxFileMgr API, reference ``box_helper_py.cc:167-216``,
``box_wrapper.cc:1326-1397``).  The reference wraps a proprietary AFS/HDFS
client; here it is the local (or mounted network) filesystem plus optional
``hadoop fs``-style pipe commands for reads (``fs_open_read``,
``fw/io/fs.h:38-97``)."""
from __future__ import annotations

import os
import shutil
import subprocess
from typing import List, Tuple


class BoxFileMgr:
    def __init__(self):
        self.inited = False

    def init(self, fs_name: str = "", fs_ugi: str = "", conf_path: str = "", expire_time: int = 0) -> bool:
        self.inited = True
        return True

    def list_dir(self, path: str) -> List[str]:
        return sorted(os.path.join(path, f) for f in os.listdir(path)) if os.path.isdir(path) else []

    def makedir(self, path: str) -> bool:
        os.makedirs(path, exist_ok=True)
        return True

    def exists(self, path: str) -> bool:
        return os.path.exists(path)

    def download(self, remote: str, local: str) -> bool:
        if os.path.isdir(remote):
            shutil.copytree(remote, local, dirs_exist_ok=True)
        else:
            os.makedirs(os.path.dirname(os.path.abspath(local)), exist_ok=True)
            shutil.copy2(remote, local)
        return True

    def upload(self, local: str, remote: str) -> bool:
        return self.download(local, remote)

    def remove(self, path: str) -> bool:
        if os.path.isdir(path):
            shutil.rmtree(path)
        elif os.path.exists(path):
            os.remove(path)
        return True

    def file_size(self, path: str) -> int:
        return os.path.getsize(path) if os.path.exists(path) else -1

    def dus(self, path: str) -> int:
        if os.path.isfile(path):
            return os.path.getsize(path)
        tot = 0
        for root, _, files in os.walk(path):
            for f in files:
                tot += os.path.getsize(os.path.join(root, f))
        return tot

    def truncate(self, path: str, size: int) -> bool:
        with open(path, "a") as f:
            f.truncate(size)
        return True

    def touch(self, path: str) -> bool:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a"):
            os.utime(path, None)
        return True

    def rename(self, src: str, dst: str) -> bool:
        os.replace(src, dst)
        return True

    def list_info(self, path: str) -> List[Tuple[str, int]]:
        return [(p, self.file_size(p)) for p in self.list_dir(path)]

    def count(self, path: str) -> int:
        return len(self.list_dir(path))

    def finalize(self):
        self.inited = False


def fs_open_read(path: str, pipe_command: str = "cat"):
    """Open a file through an optional converter pipe (``fs_open_read``)."""
    if not pipe_command or pipe_command == "cat":
        return open(path, "rb")
    p = subprocess.Popen(f"{pipe_command} < '{path}'", shell=True, stdout=subprocess.PIPE)
    return p.stdout
