"""Import shim for the package directory `multi-modal-retrieval-predict-project_amd/`.

The repo layout names the package directory with hyphens, which is not a valid Python identifier,
so `import mmr_amd` loads that directory as the package `mmr_amd` (all intra-package imports are
relative).  Nothing else lives here.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "multi-modal-retrieval-predict-project_amd")
_spec = _ilu.spec_from_file_location("mmr_amd", _os.path.join(_DIR, "__init__.py"),
                                     submodule_search_locations=[_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["mmr_amd"] = _mod
_spec.loader.exec_module(_mod)
