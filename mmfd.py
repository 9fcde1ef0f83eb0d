"""Import shim: `import mmfd` loads the package that lives in
`multimodal-misinformation-detection_amd/` (a directory name Python cannot import directly)."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_root = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "multimodal-misinformation-detection_amd")
_spec = _ilu.spec_from_file_location("mmfd", _os.path.join(_root, "__init__.py"), submodule_search_locations=[_root])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["mmfd"] = _mod
_spec.loader.exec_module(_mod)
