"""The measurement files the documents cite exist under profiles/ (CPU): DESIGN.md, README.md and
INTEGRATION.md quote numbers from `profiles/rNN_*` files, so a cited file that was renamed or never
committed would leave a number without its evidence."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cited_profiles_exist():
    text = "".join(open(os.path.join(ROOT, f)).read() for f in ("DESIGN.md", "README.md", "INTEGRATION.md"))
    # plain file names only (names written with {a,b} alternatives or * are patterns)
    names = set(re.findall(r"(r0[0-9]_[A-Za-z0-9_]+\.(?:txt|json|csv|log))", text))
    assert names, "no profile file cited"
    missing = sorted(n for n in names if not os.path.exists(os.path.join(ROOT, "profiles", n)))
    assert not missing, f"cited but not under profiles/: {missing}"
