"""Import shim: exposes the package directory ``textmae-image-compression_amd/`` as ``textmae_amd``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "textmae-image-compression_amd")
_spec = _ilu.spec_from_file_location("textmae_amd", _os.path.join(_PKG, "__init__.py"),
                                     submodule_search_locations=[_PKG])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["textmae_amd"] = _mod
_spec.loader.exec_module(_mod)
