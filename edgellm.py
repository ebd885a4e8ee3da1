"""Import alias for the ``llm-for-distributed-egde-devices_amd`` package.

The package directory carries the project name, which contains hyphens and is
therefore not a valid Python identifier.  Importing ``edgellm`` loads that
directory as a package whose canonical name is ``edgellm``; every submodule
(``edgellm.ops``, ``edgellm.models`` …) then lives under this single name, so
there is exactly one copy of each module in ``sys.modules``.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "llm-for-distributed-egde-devices_amd")
_spec = importlib.util.spec_from_file_location(
    "edgellm", os.path.join(_PKG_DIR, "__init__.py"),
    submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["edgellm"] = _mod
_spec.loader.exec_module(_mod)
