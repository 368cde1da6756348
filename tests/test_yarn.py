"""YARN integration (alluxio_amd/yarn.py; reference integration/yarn Client/ApplicationMaster) against
a fake ResourceManager REST endpoint."""
import io
import json
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer
from urllib.parse import parse_qs, urlsplit

import pytest

from alluxio_amd import yarn
from alluxio_amd.cli import main as cli


class _RM(BaseHTTPRequestHandler):
    def log_message(self, *a):
        pass

    def _send(self, code, obj=None):
        data = json.dumps(obj).encode() if obj is not None else b""
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _body(self):
        n = int(self.headers.get("Content-Length", 0))
        return json.loads(self.rfile.read(n)) if n else {}

    def do_POST(self):
        st = self.server.st
        u = urlsplit(self.path)
        if u.path.endswith("/new-application"):
            st["seq"] += 1
            return self._send(200, {"application-id": f"application_1_{st['seq']:04d}",
                                    "maximum-resource-capability": {"memory": 65536, "vCores": 32}})
        if u.path == "/ws/v1/cluster/apps":
            spec = self._body()
            st["apps"][spec["application-id"]] = dict(spec, state="RUNNING")
            return self._send(202)
        return self._send(404)

    def do_GET(self):
        st = self.server.st
        u = urlsplit(self.path)
        if u.path == "/ws/v1/cluster/apps":
            tag = parse_qs(u.query).get("applicationTags", [""])[0]
            apps = [{"id": i, "name": a["application-name"], "state": a["state"]}
                    for i, a in st["apps"].items() if tag in a["application-tags"]["tag"]]
            return self._send(200, {"apps": {"app": apps} if apps else None})
        app_id = u.path.rsplit("/", 1)[-1]
        a = st["apps"].get(app_id)
        return self._send(200, {"app": {"id": app_id, "state": a["state"]}}) if a else self._send(404)

    def do_PUT(self):
        app_id = urlsplit(self.path).path.split("/")[-2]
        self.server.st["apps"][app_id]["state"] = self._body()["state"]
        return self._send(200, {"state": "KILLED"})


@pytest.fixture
def rm():
    srv = HTTPServer(("127.0.0.1", 0), _RM)
    srv.st = {"seq": 0, "apps": {}}
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield srv
    srv.shutdown()
    srv.server_close()


def test_submit_status_stop(rm):
    url = f"http://127.0.0.1:{rm.server_address[1]}"
    out = io.StringIO()
    rc = cli.main(["yarn", "submit", "--rm", url, "--name", "c1", "--num-workers", "3", "--master-host", "m0",
                   "--home", "/opt/alluxio-amd", "--wait", "5", "-Dalluxio.worker.tieredstore.level0.dirs.path=hbm"],
                  out=out)
    assert rc == 0, out.getvalue()
    apps = rm.st["apps"]
    assert len(apps) == 4
    roles = sorted(a["application-name"] for a in apps.values())
    assert roles == ["c1-master", "c1-worker-0", "c1-worker-1", "c1-worker-2"]
    w0 = next(a for a in apps.values() if a["application-name"] == "c1-worker-0")
    gpu = w0["resource"]["resourceInformations"]["resourceInformation"][0]
    assert gpu["name"] == "yarn.io/gpu" and gpu["value"] == 1
    env = {e["key"]: e["value"] for e in w0["am-container-spec"]["environment"]["entry"]}
    assert env["ALLUXIO_MASTER_HOSTNAME"] == "m0" and env["ALLUXIO_YARN_ROLE"] == "worker"
    assert "-Dalluxio.worker.tieredstore.level0.dirs.path=hbm" in env["ALLUXIO_OPTS"]
    assert "-Dalluxio.master.hostname=m0" in env["ALLUXIO_OPTS"]
    assert w0["am-container-spec"]["commands"]["command"].startswith("/opt/alluxio-amd/bin/alluxio worker")
    m = next(a for a in apps.values() if a["application-name"] == "c1-master")
    assert "resourceInformations" not in m["resource"]
    st = yarn.status(yarn.YarnRestClient(url), "c1")
    assert len(st) == 4 and all(s["state"] == "RUNNING" for s in st)
    out = io.StringIO()
    assert cli.main(["yarn", "stop", "--rm", url, "--name", "c1"], out=out) == 0
    assert json.loads(out.getvalue())["killed"] == 4
    assert all(a["state"] == "KILLED" for a in apps.values())
    assert yarn.stop(yarn.YarnRestClient(url), "c1") == 0
