"""Packaging: the native extension is built by ``docker_dist_nn_amd._build`` (hipcc for gfx950,
g++ for the host runtime, in-tree) and shipped as package data, so ``pip install .`` and
``python setup.py build_ext --inplace`` both produce the same ``_native*.so`` the tests load."""
from setuptools import setup
from setuptools.command.build_ext import build_ext
from setuptools.command.build_py import build_py


def _native():
    from docker_dist_nn_amd._build import build

    return build()


class BuildNative(build_ext):
    def run(self):
        _native()


class BuildPyWithNative(build_py):
    def run(self):
        _native()
        super().run()


setup(
    cmdclass={"build_ext": BuildNative, "build_py": BuildPyWithNative},
    package_data={"docker_dist_nn_amd": ["_native*.so", "ops/*.json", "parallel/*.json"]},
)
