"""In-process swarm helpers for tests: stage servers in threads, registry + TCP RPC on localhost."""
import threading
import time

from src import main as M


class ServerThread:
    def __init__(self, argv):
        self.args = M.build_parser().parse_args(argv)
        self.device = M.pick_device(self.args)
        self.stop = threading.Event()
        self.ready = threading.Event()
        self.dht = self.srv = None
        self.error = None
        cfg = M.resolve_model(self.args.model)
        self.cuts = M.parse_splits(self.args.splits, cfg.num_hidden_layers)
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _on_ready(self, dht, srv):
        self.dht, self.srv = dht, srv
        self.ready.set()

    def _run(self):
        try:
            M.run_stage_server(self.args, self.device, self.cuts, self.stop, self._on_ready)
        except Exception as e:  # pragma: no cover
            self.error = e
            self.ready.set()

    def wait(self, timeout=60):
        assert self.ready.wait(timeout), "server did not start"
        if self.error:
            raise self.error
        return self

    @property
    def addr(self):
        return self.dht.get_visible_maddrs()[0]

    def kill(self):
        """Abrupt failure: stop serving without announcing anything (records just age out)."""
        if self.srv is not None:
            self.srv._stop.set()
            try:
                self.srv.loop.run(self.srv.server.shutdown(), timeout=5)
            except Exception:
                pass
        self.stop.set()

    def close(self):
        self.stop.set()
        self.thread.join(10)


def server_argv(model, splits, stage, peers="", extra=""):
    a = f"--model {model} --splits {splits} --stage {stage} --dht_port 0 --rpc_port 0 --host 127.0.0.1 " \
        f"--device cpu --kv_cache_gb 0.05 --max_sessions 16 --log_level WARNING"
    if peers:
        a += f" --dht_initial_peers {peers}"
    return (a + " " + extra).split()


def client_args(model, splits, peers, extra=""):
    a = f"--model {model} --splits {splits} --stage 0 --device cpu --dht_initial_peers {peers} " \
        f"--log_level WARNING --kv_cache_gb 0.05 --max_sessions 4"
    return M.build_parser().parse_args((a + " " + extra).split())


def wait_for(pred, timeout=20, period=0.1):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(period)
    return False
