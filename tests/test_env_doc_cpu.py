"""Every HIPSERVE_* environment variable read by the code is documented in docs/ENV.md."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]
NAME = re.compile(r"HIPSERVE_[A-Z0-9_]*[A-Z0-9]")


def _names_in_code():
    files = [ROOT / "bench.py"]
    for sub, pats in (("hipserve", ("*.py",)), ("csrc", ("*.hip", "*.cpp", "*.h"))):
        for p in pats:
            files += list((ROOT / sub).rglob(p))
    found = {}
    for f in files:
        for n in NAME.findall(f.read_text(errors="replace")):
            found.setdefault(n, str(f.relative_to(ROOT)))
    return found


def test_every_env_knob_documented():
    doc = (ROOT / "docs" / "ENV.md").read_text()
    documented = set(re.findall(r"`(HIPSERVE_[A-Z0-9_]+)`", doc))
    missing = {n: f for n, f in _names_in_code().items() if n not in documented}
    assert not missing, f"undocumented HIPSERVE_* variables (add them to docs/ENV.md): {missing}"


def test_no_stale_env_docs():
    code = _names_in_code()
    doc = (ROOT / "docs" / "ENV.md").read_text()
    stale = sorted(n for n in set(re.findall(r"`(HIPSERVE_[A-Z0-9_]+)`", doc)) if n not in code)
    assert not stale, f"docs/ENV.md lists variables no code reads: {stale}"
