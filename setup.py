"""setuptools entry: builds the gfx950 extension (mikmeans/_build.py, hipcc) before packaging.

The extension is compiled in-tree (mikmeans/_C*.so) so a source checkout, an editable
install and a wheel all load the same binary; `python -m mikmeans._build` does the
same thing by hand.
"""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildWithNative(build_py):
    def run(self):
        from mikmeans._build import build

        build(verbose=False)
        super().run()


setup(cmdclass={"build_py": BuildWithNative})
