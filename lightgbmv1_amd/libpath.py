"""Locate the native library (reference python-package/lightgbm/libpath.py).

The library is built in-tree by ``make`` (or ``__graft_entry__.build()``) into
``lightgbmv1_amd/lib/lib_lightgbmv1_amd.so``; ``LIGHTGBM_AMD_LIB`` overrides the path.
"""
import os


def find_lib_path():
    """Return the candidate paths of the native library that exist."""
    env = os.environ.get("LIGHTGBM_AMD_LIB")
    here = os.path.dirname(os.path.abspath(__file__))
    candidates = []
    if env:
        candidates.append(env)
    candidates += [
        os.path.join(here, "lib", "lib_lightgbmv1_amd.so"),
        os.path.join(here, "..", "lightgbmv1_amd", "lib", "lib_lightgbmv1_amd.so"),
    ]
    found = [os.path.abspath(p) for p in candidates if os.path.isfile(p)]
    if not found:
        raise Exception("Cannot find lib_lightgbmv1_amd.so; build it with `make -j8` in the repository root.\n"
                        "Searched:\n" + "\n".join(candidates))
    return found
