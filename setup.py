"""Build the native parts of paddlebox_amd in-tree.

  python setup.py build_ext --inplace      (PYTORCH_ROCM_ARCH=gfx950 is forced)

Two extensions:
  paddlebox_amd._pbx_hip   hand-written gfx950 HIP kernels + GPU table (torch glue)
  paddlebox_amd._pbx_host  native C++ host runtime: CPU parameter server, slot
                           dataset/parser, metrics, thread pool/channel, archive
"""
import glob
import os

os.environ["PYTORCH_ROCM_ARCH"] = "gfx950"
os.environ.setdefault("MAX_JOBS", str(min(8, os.cpu_count() or 8)))

from setuptools import setup  # noqa: E402
from torch.utils.cpp_extension import BuildExtension, CppExtension, CUDAExtension  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))


def rel(p):
    return os.path.relpath(p, ROOT)


def _drop_stale_hip_objects():
    """torch's ninja build gives hipcc no depfile, so a .hip object is rebuilt
    only when the .hip itself changes -- not when a header it includes does.
    A struct change in kernels.h (e.g. a field added to TowerArgs) then leaves
    objects compiled with the old layout next to callers built with the new
    one: kernel arguments read at shifted offsets, a GPU memory fault.  Drop
    every HIP object older than the newest header before building."""
    headers = glob.glob(os.path.join(ROOT, "csrc", "hip", "*.h")) + glob.glob(os.path.join(ROOT, "csrc", "common", "*.h"))
    if not headers:
        return
    newest = max(os.path.getmtime(h) for h in headers)
    for obj in glob.glob(os.path.join(ROOT, "build", "temp.*", "csrc", "hip", "*.o")):
        if os.path.getmtime(obj) < newest:
            os.remove(obj)


_drop_stale_hip_objects()

hip_sources = sorted(glob.glob(os.path.join(ROOT, "csrc", "hip", "*.hip"))) + sorted(
    glob.glob(os.path.join(ROOT, "csrc", "hip", "*.cpp"))
)
host_sources = sorted(glob.glob(os.path.join(ROOT, "csrc", "host", "*.cc")))

exts = [
    CUDAExtension(
        "paddlebox_amd._pbx_hip",
        [rel(p) for p in hip_sources],
        include_dirs=[os.path.join(ROOT, "csrc")],
        extra_compile_args={
            "cxx": ["-O3", "-std=c++17"],
            "nvcc": ["-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics"],
        },
    ),
]
if host_sources:
    exts.append(
        CppExtension(
            "paddlebox_amd._pbx_host",
            [rel(p) for p in host_sources],
            include_dirs=[os.path.join(ROOT, "csrc")],
            extra_compile_args=["-O3", "-std=c++17", "-fopenmp"],
            extra_link_args=["-fopenmp"],
        )
    )

setup(
    name="paddlebox_amd",
    version="0.1.0",
    packages=["paddlebox_amd"],
    ext_modules=exts,
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
