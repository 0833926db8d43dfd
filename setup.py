"""Packaging shim: the native extensions are built in-tree by
tensorflow_distributed_on_gke_amd/_build.py (ninja + hipcc --offload-arch=gfx950),
then shipped as package data (see pyproject.toml)."""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        from tensorflow_distributed_on_gke_amd import _build

        _build.build()
        super().run()


setup(cmdclass={"build_py": BuildNative})
