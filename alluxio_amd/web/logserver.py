"""Remote log server + the handler processes use to ship their logs to it.

Parity: logserver/src/main/java/alluxio/logserver/AlluxioLogServerProcess.java (accept socket
connections from processes' log appenders; one handler thread per connection) and
AlluxioLog4jSocketNode.java (route each event to ``<logs dir>/<process type>/<client host>.log``).
Events travel as newline-delimited JSON (never pickled objects), so the server executes nothing
it receives.
"""
from __future__ import annotations

import json
import logging
import os
import socket
import socketserver
import threading
import time

LOG = logging.getLogger(__name__)


class LogServer:
    def __init__(self, logs_dir: str, host: str = "127.0.0.1", port: int = 0):
        self.logs_dir = logs_dir
        os.makedirs(logs_dir, exist_ok=True)
        self._files: dict[str, object] = {}
        self._lock = threading.Lock()
        outer = self

        class Handler(socketserver.StreamRequestHandler):
            def handle(self):
                peer = self.client_address[0]
                for line in self.rfile:
                    try:
                        ev = json.loads(line)
                    except ValueError:
                        continue
                    outer.write(ev, peer)

        class Server(socketserver.ThreadingTCPServer):
            allow_reuse_address = True
            daemon_threads = True

        self.server = Server((host, port), Handler)

    @property
    def port(self) -> int:
        return self.server.server_address[1]

    def _file(self, process_type: str, host: str):
        key = f"{process_type}/{host}"
        with self._lock:
            f = self._files.get(key)
            if f is None:
                d = os.path.join(self.logs_dir, process_type.lower())
                os.makedirs(d, exist_ok=True)
                f = self._files[key] = open(os.path.join(d, f"{host}.log"), "a", buffering=1)
            return f

    def write(self, ev: dict, peer: str) -> None:
        ptype = str(ev.get("process", "unknown")).replace("/", "_") or "unknown"
        host = str(ev.get("host") or peer).replace("/", "_")
        ts = time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(ev.get("created", time.time())))
        line = f"{ts} {ev.get('level', 'INFO')} {ev.get('logger', '')} - {ev.get('msg', '')}\n"
        f = self._file(ptype, host)
        with self._lock:
            f.write(line)

    def start(self) -> int:
        threading.Thread(target=self.server.serve_forever, kwargs={"poll_interval": 0.05}, name="logserver",
                         daemon=True).start()
        return self.port

    def stop(self) -> None:
        self.server.shutdown()
        self.server.server_close()
        with self._lock:
            for f in self._files.values():
                f.close()
            self._files.clear()


class RemoteLogHandler(logging.Handler):
    """logging.Handler that ships records as JSON lines to a LogServer (reconnects lazily)."""

    def __init__(self, host: str, port: int, process_type: str):
        super().__init__()
        self.addr = (host, port)
        self.process_type = process_type
        self.hostname = socket.gethostname()
        self._sock = None
        self._lock2 = threading.Lock()

    def emit(self, record):
        try:
            ev = {"process": self.process_type, "host": self.hostname, "logger": record.name,
                  "level": record.levelname, "created": record.created, "msg": self.format(record)}
            data = (json.dumps(ev) + "\n").encode()
            with self._lock2:
                if self._sock is None:
                    self._sock = socket.create_connection(self.addr, timeout=5)
                self._sock.sendall(data)
        except OSError:
            self._sock = None

    def close(self):
        with self._lock2:
            if self._sock is not None:
                self._sock.close()
                self._sock = None
        super().close()


def attach(process_type: str, conf) -> RemoteLogHandler | None:
    """Ship this process's logs to ``alluxio.logserver.hostname:port`` when configured."""
    host = conf.get_raw("alluxio.logserver.hostname")
    if not host:
        return None
    h = RemoteLogHandler(host, conf.get_int("alluxio.logserver.port"), process_type)
    logging.getLogger().addHandler(h)
    return h


def main(argv=None) -> int:  # pragma: no cover - CLI entry
    import argparse
    from ..conf import Configuration
    ap = argparse.ArgumentParser(description="alluxio_amd log server")
    ap.add_argument("--logs-dir", default=None)
    ap.add_argument("--port", type=int, default=None)
    a = ap.parse_args(argv)
    conf = Configuration(load_site=True)
    srv = LogServer(a.logs_dir or conf.get("alluxio.logserver.logs.dir"), "0.0.0.0",
                    a.port if a.port is not None else conf.get_int("alluxio.logserver.port"))
    srv.start()
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        pass
    srv.stop()
    return 0
