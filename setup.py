"""setuptools entry: builds the gfx950 extension (mikmeans/_build.py, hipcc) before packaging.

The extension is compiled in-tree (mikmeans/_C*.so) so a source checkout, an editable
install and a wheel all load the same binary; `python -m mikmeans._build` does the
same thing by hand.  Metadata lives here (not in pyproject [project]) so the image's
setuptools 59 can build it offline.
"""
import os
import sys

from setuptools import Distribution, find_packages, setup
from setuptools.command.build_py import build_py

HERE = os.path.dirname(os.path.abspath(__file__))


class BuildWithNative(build_py):
    def run(self):
        sys.path.insert(0, HERE)
        from mikmeans._build import build

        build(verbose=False)
        super().run()


class BinaryDistribution(Distribution):
    """The package ships a compiled gfx950 extension: platform wheel, not py3-none-any."""

    def has_ext_modules(self):
        return True


setup(
    distclass=BinaryDistribution,
    name="mikmeans",
    version="0.1.0",
    description="MI355X-native k-means: gfx950 HIP MFMA kernels, RCCL data parallelism, PyTorch-ROCm",
    long_description=open(os.path.join(HERE, "README.md"), encoding="utf-8").read(),
    long_description_content_type="text/markdown",
    license="MIT",
    python_requires=">=3.10",
    packages=find_packages(include=["mikmeans", "mikmeans.*"]),
    package_data={"mikmeans": ["csrc/*.hip", "csrc/*.h", "csrc/*.cpp", "_C*.so"]},
    install_requires=["torch", "numpy", "safetensors"],
    extras_require={"test": ["pytest", "scikit-learn"]},
    entry_points={"console_scripts": ["mikmeans = mikmeans.cli:main"]},
    cmdclass={"build_py": BuildWithNative},
)
