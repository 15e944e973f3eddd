"""Run the reference's own code from its source text (TEST INFRASTRUCTURE ONLY).

Used in THIS container only, to generate golden fixtures (oracle/
gen_ref_pins.py); nothing under tests/, smoke() or bench.py imports this
module at run time, and /root/reference does not exist on the GPU box.

The reference package cannot be imported as a package here (its
``__init__`` needs gym; Optimize needs the missing ``custom_envs.models``;
utils_math needs numexpr -- ordinary ModuleNotFoundErrors).
Its hot-path functions and classes are plain Python over numpy, so this
module parses a reference file with ``ast``, keeps only the named top-level
definitions, and compiles them with the reference file's path as their code
filename into a namespace the caller fills with what their module-level
imports would have bound.  What gets executed is exactly the reference's
text for those definitions; the namespace entries are the only substitutes
and every generating script names them.
"""
import ast
import os

REFERENCE = os.environ.get('CE_REFERENCE', '/root/reference')


def _names(node):
    if isinstance(node, (ast.FunctionDef, ast.ClassDef)):
        return [node.name]
    if isinstance(node, ast.Assign):
        return [t.id for t in node.targets if isinstance(t, ast.Name)]
    return []


def load(relpath, names, namespace):
    """Execute the top-level definitions ``names`` of reference file
    ``relpath`` into ``namespace`` (a dict); returns the namespace."""
    path = os.path.join(REFERENCE, relpath)
    with open(path) as fh:
        tree = ast.parse(fh.read(), filename=path)
    wanted = set(names)
    body = [node for node in tree.body if wanted & set(_names(node))]
    found = {n for node in body for n in _names(node)}
    missing = wanted - found
    if missing:
        raise KeyError('%s defines no %s' % (relpath, sorted(missing)))
    code = compile(ast.Module(body=body, type_ignores=[]), path, 'exec')
    exec(code, namespace)   # noqa: S102 -- the reference's own definitions
    return namespace


def available():
    return os.path.isdir(os.path.join(REFERENCE, 'custom_envs'))
