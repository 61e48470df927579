"""Every file the docs cite as evidence exists: profiles/ records, scripts/ and tools/ sources named in DESIGN.md,
README.md, INTEGRATION.md and profiles/INDEX.md (a number whose record was renamed or overwritten is a claim
without its evidence). Patterns such as `profiles/r04_c*_bench.json` are not checked."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md", "profiles/INDEX.md"]
CITE = re.compile(r"\b((?:profiles|scripts|tools)/[A-Za-z0-9_.\-/]+)")


def _citations(doc):
    text = open(os.path.join(ROOT, doc)).read()
    for m in CITE.finditer(text):
        path = m.group(1).rstrip(".,;:)")
        nxt = text[m.end():m.end() + 1]
        if nxt in "*{<" or path.endswith("/") or path.endswith("_"):
            continue  # a pattern or a directory prefix, not a file
        yield path


@pytest.mark.parametrize("doc", DOCS)
def test_cited_files_exist(doc):
    missing = sorted({p for p in _citations(doc) if not os.path.exists(os.path.join(ROOT, p))})
    assert not missing, f"{doc} cites files that do not exist: {missing}"


def test_index_lists_existing_profiles():
    text = open(os.path.join(ROOT, "profiles", "INDEX.md")).read()
    names = set(re.findall(r"`((?:r0[0-9]_|pmc_)[A-Za-z0-9_.\-]+)`", text))
    missing = sorted(n for n in names if not os.path.exists(os.path.join(ROOT, "profiles", n)))
    assert not missing, f"profiles/INDEX.md lists files that do not exist: {missing}"
