"""Package metadata for ``pip wheel .`` / ``pip install .`` (release tarballs: tools/release.py).

Build the gfx950 extension in-tree first (``python -c "import __graft_entry__ as g; g.build()"``):
the wheel then carries ``alluxio_amd/_C*.so`` next to the HIP/C++ sources it was built from.
"""
import os
import re

from setuptools import Distribution, find_packages, setup

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "alluxio_amd", "__init__.py")) as f:
    VERSION = re.search(r'__version__ = "([^"]+)"', f.read()).group(1)



class _NativeDistribution(Distribution):
    """The wheel carries a prebuilt CPython extension: tag it for this interpreter/platform."""

    def has_ext_modules(self):
        return True


setup(
    distclass=_NativeDistribution,
    name="alluxio-amd",
    version=VERSION,
    description="MI355X-native data orchestration: Alluxio-compatible master/worker/client with HBM3E "
                "tiers, HIP kernels and xGMI peer transfer",
    long_description=open(os.path.join(HERE, "README.md")).read(),
    long_description_content_type="text/markdown",
    python_requires=">=3.10",
    packages=find_packages(include=["alluxio_amd", "alluxio_amd.*"]),
    package_data={"alluxio_amd": ["_C*.so", "csrc/*.cpp", "csrc/*.h", "csrc/*.hip", "web/static/webui/*"]},
    install_requires=["numpy", "grpcio", "protobuf", "torch"],
    extras_require={"table": ["pyarrow"], "web": ["fastapi", "uvicorn"], "test": ["pytest", "pytest-timeout"]},
    entry_points={"console_scripts": ["alluxio = alluxio_amd.cli.main:main"]},
    zip_safe=False,
)
