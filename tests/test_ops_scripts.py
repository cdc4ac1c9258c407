"""Deployment tooling: shell syntax, and auto_pull fast-forwarding a checkout."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = ["deploy.sh", "auto_pull.sh", "setup_auto_pull.sh"]


@pytest.mark.parametrize("name", SCRIPTS)
def test_shell_syntax(name):
    path = os.path.join(ROOT, "scripts", name)
    if not os.path.exists(path):
        pytest.skip(f"{name} absent")
    subprocess.run(["bash", "-n", path], check=True)


def _git(cwd, *args):
    env = dict(os.environ, GIT_AUTHOR_NAME="t", GIT_AUTHOR_EMAIL="t@t", GIT_COMMITTER_NAME="t",
               GIT_COMMITTER_EMAIL="t@t")
    return subprocess.run(["git", *args], cwd=cwd, check=True, capture_output=True, text=True, env=env).stdout.strip()


def test_auto_pull_fast_forwards(tmp_path):
    origin, work, dev = tmp_path / "origin.git", tmp_path / "work", tmp_path / "dev"
    _git(tmp_path, "init", "-q", "--bare", "-b", "main", str(origin))
    _git(tmp_path, "clone", "-q", str(origin), str(dev))
    (dev / "a.txt").write_text("1")
    _git(dev, "add", "a.txt")
    _git(dev, "commit", "-qm", "one")
    _git(dev, "push", "-q", "origin", "HEAD:main")
    _git(tmp_path, "clone", "-q", "-b", "main", str(origin), str(work))
    (dev / "a.txt").write_text("2")
    _git(dev, "commit", "-qam", "two")
    _git(dev, "push", "-q", "origin", "HEAD:main")
    marker = tmp_path / "restarted"
    env = dict(os.environ, ONCE="1", LOG=str(tmp_path / "pull.log"))
    subprocess.run(["bash", os.path.join(ROOT, "scripts", "auto_pull.sh"), str(work), "main", "1",
                    f"touch {marker}"], check=True, env=env, timeout=60, capture_output=True)
    assert (work / "a.txt").read_text() == "2"
    assert marker.exists()
    assert "updated" in (tmp_path / "pull.log").read_text()


def test_setup_auto_pull_dry_run():
    out = subprocess.run(["bash", os.path.join(ROOT, "scripts", "setup_auto_pull.sh"), ROOT, "main", "30"],
                         check=True, capture_output=True, text=True, env=dict(os.environ, DRY_RUN="1")).stdout
    assert "ExecStart=/bin/bash" in out and "auto_pull.sh" in out and " main 30 " in out
