"""Import shim: `import pamd` loads the package directory
`partitionedarrays.jl_amd/` (its name is not a Python identifier)."""
import importlib.util
import os
import sys

_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "partitionedarrays.jl_amd")
_spec = importlib.util.spec_from_file_location("pamd", os.path.join(_dir, "__init__.py"),
                                               submodule_search_locations=[_dir])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["pamd"] = _mod
_spec.loader.exec_module(_mod)
