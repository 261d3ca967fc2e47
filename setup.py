"""Packaging: ``pip install -e .`` / ``python setup.py build_ext --inplace``.

The native libraries are built in-tree by tools/build_native.py (hipcc --offload-arch=gfx950 for
csrc/kernels/*.hip, g++ for the csrc/runtime/*.cpp host runtime) and shipped as package data; the
Python side loads them with ctypes (no torch C++ extension ABI coupling).
"""
import os
import sys

from setuptools import Command, find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


def _build_native(force=False):
    sys.path.insert(0, ROOT)
    from tools.build_native import build
    build(force=force)


class BuildNative(Command):
    description = "build libdtm_kernels.so (gfx950 HIP) and libdtm_runtime.so in-tree"
    user_options = [("force", "f", "rebuild everything")]

    def initialize_options(self):
        self.force = False

    def finalize_options(self):
        pass

    def run(self):
        _build_native(bool(self.force))


class BuildPy(build_py):
    def run(self):
        _build_native()
        super().run()


class BuildExtInplace(BuildNative):
    description = "alias of build_native (in-tree build)"
    user_options = BuildNative.user_options + [("inplace", "i", "ignored: the build is always in-tree")]

    def initialize_options(self):
        super().initialize_options()
        self.inplace = True


setup(
    name="distributed_tensorflow_models_amd",
    version="0.1.0",
    description="MI355X-native distributed CNN training (TF-slim/tf.train compatible facade, HIP kernels, RCCL)",
    packages=find_packages(include=["distributed_tensorflow_models_amd", "distributed_tensorflow_models_amd.*"]),
    package_data={"distributed_tensorflow_models_amd": ["_native/*.so"]},
    python_requires=">=3.10",
    install_requires=["torch", "numpy"],
    cmdclass={"build_native": BuildNative, "build_py": BuildPy, "build_ext": BuildExtInplace},
    entry_points={"console_scripts": [
        "dtm-launch=distributed_tensorflow_models_amd.parallel.launcher:main",
        "dtm-ssp-clock=distributed_tensorflow_models_amd.parallel.ssp:main",
    ]},
)
