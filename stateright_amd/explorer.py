"""Explorer over the GPU checker (§8f rank 3): the reference's HTTP routes and JSON shapes
(src/checker/explorer.rs:12-22,118-240) served by the standard library, with every answer computed
through the engine's C ABI (sr_gpu_bfs_explore walks a fingerprint path on the engine's host copy
of the model; counts and discoveries come from the running GPU check).

    GET /.status                      {"done", "model", "state_count", "unique_state_count",
                                       "properties": [[expectation, name, "fp/fp/..." | null]],
                                       "recent_path"}
    GET /.states/<fp>/<fp>/...        [{"action", "outcome", "state", "fingerprint"}, ...]
    GET /                             a small UI over the two routes

Fingerprints are the engine's (models.hpp `fingerprint<W>`), not ahash values; states are the
models' canonical descriptions. `recent_path`: the reference samples the path of a recently popped
state through a visitor every 4 s (explorer.rs:57-89); the GPU pops a whole level per launch, so
it reports the shortest discovery path's actions once the check is done (null before).
"""
import http.server
import json
import threading
from urllib.parse import unquote

EXPECTATIONS = {0: "Always", 1: "Eventually", 2: "Sometimes"}

INDEX = """<!doctype html>
<html><head><meta charset="utf-8"><title>Stateright Explorer (MI355X engine)</title>
<style>body{font-family:monospace;margin:1.5em} a{cursor:pointer;color:#06c} li{margin:.3em 0}
pre{background:#f4f4f4;padding:.4em}</style></head>
<body><h2>Stateright Explorer &mdash; MI355X breadth-first engine</h2>
<div id="status"></div><h3>Path</h3><ol id="path"></ol><h3>Next steps</h3><ul id="steps"></ul>
<script>
let path = [];
function fps() { return path.map(p => p.fingerprint); }
async function refresh() {
  const st = await (await fetch('/.status')).json();
  document.getElementById('status').innerHTML =
    `<p>done=${st.done} states=${st.state_count} unique=${st.unique_state_count}</p><ul>` +
    st.properties.map(p => `<li>${p[0]} "${p[1]}": ` + (p[2] ? `<a onclick="go('${p[2]}')">discovery</a>` : 'none') +
    '</li>').join('') + '</ul>';
  const views = await (await fetch('/.states/' + fps().join('/'))).json();
  document.getElementById('path').innerHTML = path.map((p, i) =>
    `<li><a onclick="back(${i})">${p.action || 'init'}</a><pre>${p.state}</pre></li>`).join('');
  document.getElementById('steps').innerHTML = views.map((v, i) => v.fingerprint ?
    `<li><a onclick='step(${JSON.stringify(v)})'>${v.action || 'init'}</a><pre>${v.state}</pre></li>` :
    `<li>${v.action} (ignored)</li>`).join('');
}
function step(v) { path.push(v); refresh(); }
function back(i) { path = path.slice(0, i + 1); refresh(); }
async function go(enc) {
  const fs = enc.split('/'); path = [];
  for (let i = 0; i < fs.length; i++) {
    const views = await (await fetch('/.states/' + fs.slice(0, i).join('/'))).json();
    const v = views.find(v => v.fingerprint === fs[i]); if (!v) break; path.push(v);
  }
  refresh();
}
setInterval(refresh, 4000); refresh();
</script></body></html>
"""


class Explorer:
    """Serves the Explorer routes for `checker` (a running or finished GpuBfsChecker)."""

    def __init__(self, checker, address=("127.0.0.1", 3000), model_name=None):
        self.checker = checker
        self.model_name = model_name or type(checker.model()).__name__
        self._lock = threading.Lock()
        ex = self

        class Handler(http.server.BaseHTTPRequestHandler):
            def log_message(self, *args):
                pass

            def _send(self, code, body, ctype="application/json"):
                data = body.encode() if isinstance(body, str) else body
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                path = unquote(self.path.split("?", 1)[0])
                if path == "/.status":
                    return self._send(200, json.dumps(ex.status()))
                if path.startswith("/.states"):
                    code, body = ex.states(path[len("/.states"):])
                    return self._send(code, json.dumps(body) if code == 200 else body,
                                      "application/json" if code == 200 else "text/plain")
                if path in ("/", "/index.htm"):
                    return self._send(200, INDEX, "text/html")
                return self._send(404, "not found", "text/plain")

        self._server = http.server.ThreadingHTTPServer(address, Handler)
        self.url = f"http://{self._server.server_address[0]}:{self._server.server_address[1]}"
        self._thread = None

    # --- routes (src/checker/explorer.rs:133-240) -------------------------------------------------
    def status(self):
        c = self.checker
        with self._lock:
            done = c.is_done() or not c._lib.sr_gpu_bfs_is_running(c._h)
            props = []
            recent = None
            for name, exp in c.properties():
                enc = None
                if done:
                    fps = c.discovery_fingerprints(name)
                    if fps:
                        enc = "/".join(str(f) for f in fps)
                        p = c.discovery(name)
                        if recent is None or len(p) < len(recent):
                            recent = p
                props.append([EXPECTATIONS[int(exp)], name, enc])
            return {"done": c.is_done(), "model": self.model_name, "state_count": c.state_count(),
                    "unique_state_count": c.unique_state_count(), "properties": props,
                    "recent_path": None if recent is None else "[" + ", ".join(recent.into_actions()) + "]"}

    def states(self, fingerprints_str):
        """(status code, body) of the `states` route for '/<fp>/<fp>...' (explorer.rs:159-240)."""
        s = fingerprints_str[:-1] if fingerprints_str.endswith("/") else fingerprints_str
        parts = s.split("/")
        fps = []
        for p in parts[1:]:
            try:
                fps.append(int(p))
            except ValueError:
                break
        if len(fps) + 1 != len(parts) and s != "":
            return 404, f"Unable to parse fingerprints {s}"
        with self._lock:
            views = self.checker.explore(fps)
        if views is None:
            return 404, f"Unable to find state following fingerprints {s}"
        out = []
        for action, state, fp in views:
            v = {}
            if action is not None:
                v["action"] = action
            if state is not None:
                if action is not None:
                    v["outcome"] = str(state)  # format_step's default: the next state (lib.rs:180-185)
                v["state"] = str(state)
                v["fingerprint"] = str(fp)
            out.append(v)
        return 200, out

    # --- server lifecycle ---------------------------------------------------------------------------
    def start(self):
        self._thread = threading.Thread(target=self._server.serve_forever, daemon=True)
        self._thread.start()
        return self

    def serve_forever(self):
        self._server.serve_forever()

    def shutdown(self):
        if self._thread is not None:
            self._server.shutdown()
            self._thread.join()
            self._thread = None
        self._server.server_close()
