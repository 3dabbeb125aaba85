"""Import shim: the package lives in ``pybullet-gym_amd/`` (a directory name Python
cannot import directly); this module loads it under the name ``pybulletgym_amd``."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pybullet-gym_amd")
_spec = importlib.util.spec_from_file_location(
    "pybulletgym_amd", os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["pybulletgym_amd"] = _mod
_spec.loader.exec_module(_mod)
