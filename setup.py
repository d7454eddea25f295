"""pip-installable package (reference python-package/setup.py): building the wheel runs the
native build (make; hipcc for gfx950) and ships lib_lightgbmv1_amd.so + the CLI inside the
package.

    pip install .                       # or: python setup.py bdist_wheel
    LGBM_AMD_ARCH=gfx950 pip install .  # GPU target (default gfx950)
"""
import os
import subprocess

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(build_py):
    """Compile the native library in-tree before the Python files are collected."""

    def run(self):
        jobs = str(min(16, os.cpu_count() or 8))
        arch = os.environ.get("LGBM_AMD_ARCH", "gfx950")
        subprocess.check_call(["make", "-j" + jobs, "ARCH=" + arch], cwd=ROOT)
        super().run()


class NativeDistribution(Distribution):
    """The wheel carries a native library: platform-specific tags."""

    def has_ext_modules(self):
        return True


setup(
    name="lightgbmv1_amd",
    distclass=NativeDistribution,
    version="3.0.0.99",
    description="MI355X-native gradient boosting (LightGBM-compatible API, HIP/CDNA4 tree learner)",
    packages=find_packages(include=["lightgbmv1_amd", "lightgbmv1_amd.*"]),
    package_data={"lightgbmv1_amd": ["lib/lib_lightgbmv1_amd.so", "lib/lightgbm"]},
    include_package_data=True,
    install_requires=["numpy", "scipy"],
    extras_require={"sklearn": ["scikit-learn"], "pandas": ["pandas"]},
    python_requires=">=3.8",
    cmdclass={"build_py": BuildNative},
    zip_safe=False,
)
