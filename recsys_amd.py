"""Importable alias for the package directory
`llm-driven_content-based-feature_recommendation_system_amd/` (whose name is not a Python
identifier). `import recsys_amd` replaces this module with that package, so
`recsys_amd.tower_code.v1_refine_usertower` etc. resolve to the real sub-modules."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "llm-driven_content-based-feature_recommendation_system_amd")
_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_PKG_DIR, "__init__.py"),
                                               submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
