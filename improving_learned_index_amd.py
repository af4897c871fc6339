"""Import shim: exposes the package directory ``improving-learned-index_amd/`` (whose
name is not a Python identifier) as the package ``improving_learned_index_amd``.
``python -m improving_learned_index_amd.<module>`` works through it."""
import importlib.util as _u
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "improving-learned-index_amd")
_spec = _u.spec_from_file_location(__name__, _os.path.join(_dir, "__init__.py"),
                                   submodule_search_locations=[_dir])
_mod = _u.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
