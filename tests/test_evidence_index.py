"""profiles/INDEX.md and DESIGN.md cite measurement files by name; every cited
file must exist, so the evidence a number rests on cannot silently go missing."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILES = os.path.join(ROOT, 'profiles')


def _cited(path, pattern):
    with open(path) as f:
        text = f.read()
    return sorted(set(re.findall(pattern, text)))


def _exists(name):
    """A cited measurement file: in profiles/, or superseded (rounds 1-4) in
    profiles/archive/ (kept in history, off the GPU push)."""
    return any(os.path.exists(os.path.join(PROFILES, d, name)) for d in ('', 'archive'))


def test_profiles_index_cites_existing_files():
    names = _cited(os.path.join(PROFILES, 'INDEX.md'), r'`([A-Za-z0-9_.]+\.(?:jsonl|json|csv|txt))`')
    assert names
    missing = [n for n in names if not _exists(n)]
    assert not missing, missing


def test_design_cites_existing_profiles():
    names = _cited(os.path.join(ROOT, 'DESIGN.md'), r'profiles/((?:archive/)?[A-Za-z0-9_.]+\.(?:jsonl|json|csv|txt))')
    assert names
    missing = [n for n in names if not os.path.exists(os.path.join(PROFILES, n))]
    assert not missing, missing


def test_cited_scripts_exist():
    names = set()
    for doc in ('DESIGN.md', 'README.md', os.path.join('profiles', 'INDEX.md')):
        names |= set(_cited(os.path.join(ROOT, doc), r'scripts/((?:archive/)?[A-Za-z0-9_.]+\.(?:sh|py|hip))'))
    assert names
    missing = [n for n in names if not os.path.exists(os.path.join(ROOT, 'scripts', n))]
    assert not missing, missing
