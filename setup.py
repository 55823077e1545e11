"""Packaging: the ``rss-simulator`` console script of the reference (its ``setup.py:15-17``)
bound to this package, plus the import-compatible ``rss_simulator`` package.

``build_py`` builds the in-tree gfx950 library first when it is missing (the same make
step as ``__graft_entry__.build()``), and the wheel carries it as package data:
``rss_simulator_nvidia_amd/_native.py`` loads it from beside itself.

    pip install --no-build-isolation .      (offline: setuptools / wheel from the image)
"""
import os
import subprocess

from setuptools import setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(ROOT, "rss_simulator_nvidia_amd", "librss_toeplitz.so")


class BuildWithLibrary(build_py):
    def run(self):
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "rss_simulator_nvidia_amd",
                                                             "csrc")], check=True)
        super().run()


setup(
    name="rss-simulator-nvidia-amd",
    version="0.1.0",
    description="MI355X-native RSS Toeplitz hashing engine behind the rss-simulator CLI",
    license="MIT",
    python_requires=">=3.8",
    packages=["rss_simulator_nvidia_amd", "rss_simulator_nvidia_amd.arg_parse_types",
              "rss_simulator", "rss_simulator.arg_parse_types"],
    package_data={"rss_simulator_nvidia_amd": ["librss_toeplitz.so"]},
    install_requires=["numpy", "pandas", "matplotlib"],
    entry_points={"console_scripts": ["rss-simulator=rss_simulator_nvidia_amd.main:main"]},
    cmdclass={"build_py": BuildWithLibrary},
)
