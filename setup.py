"""Wheel build: compiles the gfx950 kernel library and the host library in-tree
(hivemall_amd/_build.py: hipcc --offload-arch=gfx950, g++ -O3 -fopenmp) before the package
files are collected, so the wheel carries hivemall_amd/_lib/*.so.

    pip wheel --no-build-isolation --no-deps .
"""
from setuptools import find_packages, setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution


class BuildNative(build_py):
    def run(self):
        import importlib.util
        import os

        spec = importlib.util.spec_from_file_location(
            "_hm_build", os.path.join(os.path.dirname(os.path.abspath(__file__)), "hivemall_amd", "_build.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.build_all(verbose=False)
        super().run()


class NativeDistribution(Distribution):
    """The wheel carries gfx950 / x86-64 shared objects: a platform wheel, not py3-none-any."""

    def has_ext_modules(self):
        return True


setup(
    name="hivemall-amd",
    version="0.1.0",
    description="MI355X-native (gfx950) classical ML engine with Apache Hivemall's SQL function surface",
    long_description=open("README.md").read(),
    long_description_content_type="text/markdown",
    license="Apache-2.0",
    python_requires=">=3.10",
    packages=find_packages(include=["hivemall_amd", "hivemall_amd.*"]),
    package_data={"hivemall_amd": ["_lib/*.so"]},
    install_requires=["torch", "numpy", "pandas", "pyarrow"],
    entry_points={"console_scripts": ["hivemall-sql = hivemall_amd.sql.__main__:main"]},
    cmdclass={"build_py": BuildNative},
    distclass=NativeDistribution,
)
