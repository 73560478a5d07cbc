"""tfkctl: kubectl-style CLI for the tfk control plane.

    python -m tensorflow_k8s_amd.control.tfkctl apply -f deploy/examples/mnist-lenet-cpu.yaml
    python -m tensorflow_k8s_amd.control.tfkctl get tfjobs
    python -m tensorflow_k8s_amd.control.tfkctl describe tfjob mnist
    python -m tensorflow_k8s_amd.control.tfkctl logs mnist-worker-0
    python -m tensorflow_k8s_amd.control.tfkctl wait tfjob mnist --timeout 600
    python -m tensorflow_k8s_amd.control.tfkctl delete tfjob mnist
    python -m tensorflow_k8s_amd.control.tfkctl cluster --gpus 8     # run the all-in-one control plane
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import yaml

from .client import ALIASES, BIN, ApiError, TfkClient, tfjob_condition


def _load_docs(path: str):
    text = sys.stdin.read() if path == "-" else open(path).read()
    if path.endswith(".json"):
        d = json.loads(text)
        return d if isinstance(d, list) else [d]
    return [d for d in yaml.safe_load_all(text) if d]


def _age(ts: str | None) -> str:
    if not ts:
        return "-"
    try:
        t = time.mktime(time.strptime(ts[:19], "%Y-%m-%dT%H:%M:%S")) - time.timezone
        s = int(time.time() - t)
    except ValueError:
        return "-"
    return f"{s}s" if s < 120 else (f"{s // 60}m" if s < 7200 else f"{s // 3600}h")


def _table(rows, header):
    w = [max(len(str(r[i])) for r in rows + [header]) for i in range(len(header))]
    lines = ["   ".join(str(h).ljust(w[i]) for i, h in enumerate(header))]
    lines += ["   ".join(str(c).ljust(w[i]) for i, c in enumerate(r)) for r in rows]
    return "\n".join(lines)


def cmd_get(c: TfkClient, a):
    plural = ALIASES.get(a.resource, a.resource)
    items = [c.get(plural, a.name, a.namespace)] if a.name else c.list(plural, None if a.all_namespaces else a.namespace,
                                                                      a.selector or "")
    if a.output == "json":
        print(json.dumps(items[0] if a.name else {"items": items}, indent=2))
        return
    if a.output == "yaml":
        print(yaml.safe_dump(items[0] if a.name else {"items": items}, sort_keys=False))
        return
    if plural == "tfjobs":
        rows = [(i["metadata"]["name"], tfjob_condition(i) or "-", _age(i["metadata"].get("creationTimestamp")))
                for i in items]
        print(_table(rows, ("NAME", "STATE", "AGE")))
    elif plural == "pods":
        rows = []
        for i in items:
            cs = i.get("status", {}).get("containerStatuses", [])
            rows.append((i["metadata"]["name"], i.get("status", {}).get("phase", "Pending"),
                         sum(x.get("restartCount", 0) for x in cs), i.get("spec", {}).get("nodeName", "<none>"),
                         i["metadata"].get("annotations", {}).get("tfk.io/gpu-ids", ""),
                         _age(i["metadata"].get("creationTimestamp"))))
        print(_table(rows, ("NAME", "STATUS", "RESTARTS", "NODE", "GPUS", "AGE")))
    elif plural == "events":
        rows = [(i.get("type"), i.get("reason"), i.get("involvedObject", {}).get("name"), i.get("message", "")[:80])
                for i in items]
        print(_table(rows, ("TYPE", "REASON", "OBJECT", "MESSAGE")))
    else:
        print(_table([(i["metadata"]["name"], _age(i["metadata"].get("creationTimestamp"))) for i in items],
                     ("NAME", "AGE")))


def cmd_describe(c: TfkClient, a):
    plural = ALIASES.get(a.resource, a.resource)
    obj = c.get(plural, a.name, a.namespace)
    print(yaml.safe_dump(obj, sort_keys=False))
    evs = [e for e in c.list("events", a.namespace) if e.get("involvedObject", {}).get("name") == a.name]
    if evs:
        print("Events:")
        for e in evs:
            print(f"  {e.get('type'):8s} {e.get('reason'):26s} {e.get('message')}")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="tfkctl")
    ap.add_argument("--server", default=os.environ.get("TFK_APISERVER", "http://127.0.0.1:8080"))
    ap.add_argument("-n", "--namespace", default="default")
    ap.add_argument("--token", default=None, help="bearer token (kubectl --token)")
    ap.add_argument("--certificate-authority", default=None, help="CA bundle for an https:// server")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("apply"); p.add_argument("-f", "--filename", required=True)
    p = sub.add_parser("create"); p.add_argument("-f", "--filename", required=True)
    p = sub.add_parser("get"); p.add_argument("resource"); p.add_argument("name", nargs="?")
    p.add_argument("-o", "--output", default="table"); p.add_argument("-l", "--selector")
    p.add_argument("-A", "--all-namespaces", action="store_true")
    p = sub.add_parser("describe"); p.add_argument("resource"); p.add_argument("name")
    p = sub.add_parser("delete"); p.add_argument("resource"); p.add_argument("name")
    p = sub.add_parser("logs"); p.add_argument("pod"); p.add_argument("--tail", type=int); p.add_argument("-f", "--follow", action="store_true")
    p = sub.add_parser("wait"); p.add_argument("resource"); p.add_argument("name"); p.add_argument("--timeout", type=float, default=600)
    p = sub.add_parser("crd")
    p = sub.add_parser("cluster"); p.add_argument("--gpus", type=int, default=-1); p.add_argument("--port", type=int, default=8080)
    p.add_argument("--root-dir", default="/tmp/tfk-kubelet")
    a = ap.parse_args(argv)
    c = TfkClient(a.server, token=a.token, ca=a.certificate_authority)
    try:
        if a.cmd in ("apply", "create"):
            for d in _load_docs(a.filename):
                o = c.apply(d, a.namespace) if a.cmd == "apply" else c.create(d, a.namespace)
                print(f"{o['kind'].lower()}/{o['metadata']['name']} {'configured' if a.cmd == 'apply' else 'created'}")
        elif a.cmd == "get":
            cmd_get(c, a)
        elif a.cmd == "describe":
            cmd_describe(c, a)
        elif a.cmd == "delete":
            c.delete(ALIASES.get(a.resource, a.resource), a.name, a.namespace)
            print(f"{a.resource}/{a.name} deleted")
        elif a.cmd == "logs":
            seen = 0
            while True:
                text = c.logs(a.pod, a.namespace, a.tail)
                sys.stdout.write(text[seen:])
                sys.stdout.flush()
                seen = len(text)
                if not a.follow:
                    break
                ph = c.get("pods", a.pod, a.namespace).get("status", {}).get("phase")
                if ph in ("Succeeded", "Failed"):
                    sys.stdout.write(c.logs(a.pod, a.namespace)[seen:])
                    break
                time.sleep(1)
        elif a.cmd == "wait":
            j = c.wait_tfjob(a.name, a.namespace, timeout=a.timeout)
            print(f"tfjob/{a.name} {tfjob_condition(j)}")
            return 0 if tfjob_condition(j) == "Succeeded" else 1
        elif a.cmd == "crd":
            print(json.dumps(c.get("customresourcedefinitions", "tfjobs.kubeflow.org", None), indent=2))
        elif a.cmd == "cluster":
            return subprocess.call([os.path.join(BIN, "tfk-cluster"), "--port", str(a.port), "--gpus", str(a.gpus),
                                    "--root-dir", a.root_dir])
    except ApiError as e:
        print(f"Error from server: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
