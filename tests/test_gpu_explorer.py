"""Explorer over the GPU checker (src/checker/explorer.rs): the reference's route tests restated
(explorer.rs:248-285 can_init / can_next / err_for_invalid_fingerprint, 370-416 status) over HTTP
against a running server. Fingerprints are the engine's own (the reference's are ahash values),
so the tests navigate with the fingerprints the server itself returns."""
import json
import urllib.error
import urllib.request

import pytest

pytestmark = pytest.mark.gpu
sr = pytest.importorskip("stateright_amd")


def get(ex, path):
    try:
        with urllib.request.urlopen(ex.url + path, timeout=30) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


@pytest.fixture
def clock():
    ex = sr.BinaryClock().checker().serve(("127.0.0.1", 0), block=False)
    ex.checker.join()
    yield ex
    ex.shutdown()


def test_can_init(clock):
    code, views = get(clock, "/.states/")
    assert code == 200
    assert [v["state"] for v in views] == ["(0,)", "(1,)"]  # init order (explorer.rs:251-254)
    assert all("action" not in v and "outcome" not in v for v in views)


def test_can_next(clock):
    _, views = get(clock, "/.states")
    fp = {v["state"]: v["fingerprint"] for v in views}
    code, nxt = get(clock, f"/.states/{fp['(1,)']}/{fp['(0,)']}")  # 1 -> GoLow -> 0, then its steps
    assert code == 200
    assert nxt == [{"action": "GoHigh", "outcome": "(1,)", "state": "(1,)", "fingerprint": fp["(1,)"]}]


def test_err_for_invalid_fingerprint(clock):
    assert get(clock, "/.states/one/two/three") == (404, "Unable to parse fingerprints /one/two/three")
    assert get(clock, "/.states/1/2/3") == (404, "Unable to find state following fingerprints /1/2/3")


def test_status_and_discovery_navigation():
    ex = sr.TwoPhaseSys(3).checker().serve(("127.0.0.1", 0), block=False)
    try:
        ex.checker.join()
        code, st = get(ex, "/.status")
        assert code == 200 and st["done"] is True
        assert (st["state_count"], st["unique_state_count"]) == (1146, 288)
        props = {name: (exp, enc) for exp, name, enc in st["properties"]}
        assert props["consistent"] == ("Always", None)
        assert props["abort agreement"][0] == "Sometimes" and props["abort agreement"][1]
        assert st["recent_path"].startswith("[")
        # follow the encoded discovery path through the states route: every fingerprint is a step
        fps = props["commit agreement"][1].split("/")
        for i in range(1, len(fps)):
            code, views = get(ex, "/.states/" + "/".join(fps[:i]))
            assert code == 200 and fps[i] in [v.get("fingerprint") for v in views]
        with urllib.request.urlopen(ex.url + "/", timeout=30) as r:
            assert r.status == 200 and b"Explorer" in r.read()
    finally:
        ex.shutdown()


def test_ignored_actions_are_listed():
    # the sliding puzzle lists all four slides; impossible ones are "Action ignored" views
    from stateright_amd import build
    from stateright_amd.plugin import Plugin
    pl = Plugin(build.plugin_path("sliding_puzzle"), "sliding_puzzle")
    c = pl.model(1, 2, 3, 4, 5, 6, 8, 7, 0).checker().spawn_bfs()
    c.join()
    (init,) = c.explore([])
    views = c.explore([init[2]])
    assert [v[0] for v in views] == ["Down", "Up", "Right", "Left"]
    assert [v[1] is not None for v in views] == [True, False, True, False]  # empty cell bottom-right
