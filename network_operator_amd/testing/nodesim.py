"""A simulated Kubernetes node for the fake API server: kubelet + NFD worker, real agent.

``FakeApiServer`` already plays the DaemonSet controller (one Pod per matching node, Ready
condition from ``set_agent_ready``).  ``SimNode`` plays what runs *on* the node:

* **kubelet** -- for every Pod bound to this node it starts the DaemonSet's container as a local
  process: the real ``discover`` binary with the container's ``args`` and ``NODE_NAME`` from the
  downward API.  hostPath volumes are mapped under ``host_root`` and every argument that names a
  path under a mountPath is rewritten to the mapped directory.  The container's exec
  ``readinessProbe`` runs every ``probe_period`` seconds and drives the Pod's Ready condition.
  A process that exits is restarted with backoff (``restartPolicy: Always``).  A changed pod
  template restarts the agent (rolling update, one node).  When the Pod goes away the agent gets
  SIGTERM and ``terminationGracePeriodSeconds`` before SIGKILL.
* **NFD worker** -- the mapped ``features.d`` directory is scanned every ``nfd_period`` seconds
  and its ``name=value`` lines become Node labels, added and removed as the files change (NFD's
  local feature source).

Jobs pinned to the node (the fabric validation Jobs) run once, their image mapped to a local
command by ``job_images``, and their exit status becomes the Job's status.  Init containers
(the host-nic driver container) run to completion, in order, before the agent
starts; their images are mapped to local commands by ``init_images`` (an unmapped image fails
like an image that cannot be pulled).  Not simulated: image pulls, and the probes'
``initialDelaySeconds`` / ``periodSeconds`` (``probe_period`` replaces both, so the control plane
is measured rather than probe timers).  The node's NICs are whatever its network namespace
holds: the calling process's, or ``netns`` (a ``NetnsHolder``) for the other nodes of a fabric;
``testing/e2e.py`` builds veths to a synthetic switch.

The reference's only end-to-end test deploys the operator into kind and checks that the
controller pod runs (reference test/e2e/e2e_test.go:51-120); it never runs an agent.
"""

from __future__ import annotations

import asyncio
import copy
import json
import logging
import os
import signal
import subprocess
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional, Tuple

from .. import discovery
from ..operator import kube
from ..operator.reconciler import CLEANUP_APP
from ..utils.paths import native_bin

log = logging.getLogger("nodesim")


@dataclass
class _Container:
    pod: Tuple[str, str]            # (namespace, pod name)
    daemonset: str                  # "<ns>/<name>"
    template: str                   # JSON of the pod template spec it was started from
    argv: List[str]
    probe: Optional[List[str]]
    env: Dict[str, str]
    grace_s: float
    log_path: Path
    proc: Optional[subprocess.Popen] = None
    restarts: int = 0
    next_start: float = 0.0
    backoff: float = 0.1
    ready: bool = False
    started_at: List[float] = field(default_factory=list)
    inits: List[dict] = field(default_factory=list)  # {"name", "image", "argv"} in order
    inits_done: bool = False
    log_start: int = 0               # size of the log file when the current run started
    fallback_to_logs: bool = False   # terminationMessagePolicy: FallbackToLogsOnError


class SimNode:
    def __init__(self, fake, name: str, labels: Dict[str, str], host_root: Path, sysfs_root: Optional[Path] = None,
                 probe_period: float = 0.02, nfd_period: float = 0.01, env: Optional[Dict[str, str]] = None,
                 init_images: Optional[Dict[str, List[str]]] = None, netns=None,
                 job_images: Optional[Dict[str, List[str]]] = None, agent_arg_overrides: Optional[Dict[str, str]] = None):
        self.fake, self.name = fake, name
        # "--flag" -> value replacing the DaemonSet's own (tests shorten e.g. --wait=90s)
        self.agent_arg_overrides = dict(agent_arg_overrides or {})
        self.base_labels = dict(labels)
        self.host_root = Path(host_root)
        self.sysfs_root = sysfs_root
        self.probe_period, self.nfd_period = probe_period, nfd_period
        self.extra_env = dict(env or {})
        self.init_images = dict(init_images or {})
        # hostNetwork pods join the node's network namespace: None = this process's, else a
        # testing.netns.NetnsHolder of another simulated node.
        self.netns = netns
        self.init_runs: List[dict] = []   # {"pod", "name", "rc", "t_start", "t_end"}
        # Jobs pinned to this node (spec.template.spec.nodeName): image -> command, run once each,
        # their exit status recorded on the Job (the fabric validation Jobs).
        self.job_images = dict(job_images or {})
        self.job_runs: List[dict] = []    # {"job", "rc", "t_start", "t_end"}
        self._jobs_started: set = set()
        self.containers: Dict[Tuple[str, str], _Container] = {}
        self.features: Dict[str, str] = {}
        self.exited: List[dict] = []      # {"pod", "rc", "log"} of every agent process that ended
        self._tasks: List[asyncio.Task] = []
        self._stop = asyncio.Event()

    # -- paths ---------------------------------------------------------------------------------
    def host_path(self, path: str) -> Path:
        """Where a host path of the simulated node lives in this process's filesystem."""
        return self.host_root / path.lstrip("/")

    @staticmethod
    def _mounts(pod_spec: dict, container: dict, pod: str = "") -> List[Tuple[str, str]]:
        """(mountPath, host path) of the container's hostPath mounts, and of its emptyDir mounts
        (a per-Pod directory, as the kubelet's), longest mountPath first."""
        vols = {v["name"]: v["hostPath"]["path"] for v in pod_spec.get("volumes") or [] if "hostPath" in v}
        vols.update({v["name"]: f"/var/lib/kubelet/pods/{pod or 'pod'}/volumes/{v['name']}"
                     for v in pod_spec.get("volumes") or [] if "emptyDir" in v})
        out = [(m["mountPath"].rstrip("/") or "/", vols[m["name"]]) for m in container.get("volumeMounts") or []
               if m.get("name") in vols]
        return sorted(out, key=lambda x: -len(x[0]))

    def _rewrite(self, value: str, mounts: List[Tuple[str, str]]) -> str:
        for mp, hp in mounts:
            if value == mp or value.startswith(mp + "/"):
                return str(self.host_path(hp)) + value[len(mp):]
        return value

    def _rewrite_arg(self, arg: str, mounts) -> str:
        if arg.startswith("--") and "=" in arg:
            k, v = arg.split("=", 1)
            return f"{k}={self._rewrite(v, mounts)}"
        return self._rewrite(arg, mounts)

    def _agent_argv(self, cmd: List[str], mounts) -> List[str]:
        # The image's entrypoint (and the probe's absolute binary path) is the agent binary.
        argv = [str(native_bin("discover"))] + [self._rewrite_arg(a, mounts) for a in cmd]
        for k, v in self.agent_arg_overrides.items():
            argv = [a for a in argv if a != k and not a.startswith(k + "=")] + [f"{k}={v}"]
        # The agent's built-in default label directory is a container path: name it explicitly.
        if not any(a.startswith("--nfd-features-dir") for a in argv):
            feat = self._rewrite(discovery.LABEL_FEATURES_DIR.rstrip("/"), mounts)
            argv.append(f"--nfd-features-dir={feat}/")
        return argv

    # -- kubelet ---------------------------------------------------------------------------------
    def _spec_for(self, pod: dict) -> Optional[_Container]:
        ns, pname = pod["metadata"].get("namespace", ""), pod["metadata"]["name"]
        ref = next((r for r in pod["metadata"].get("ownerReferences") or [] if r.get("kind") == "DaemonSet"), None)
        if ref is None:
            return None
        ds = self.fake.get_object(kube.DAEMONSETS, ref["name"], ns)
        if ds is None:
            return None
        spec = ds["spec"]["template"]["spec"]
        c = spec["containers"][0]
        mounts = self._mounts(spec, c, pname)
        for _, hp in mounts:  # hostPath type DirectoryOrCreate
            self.host_path(hp).mkdir(parents=True, exist_ok=True)
        env = {}
        for e in c.get("env") or []:
            if "value" in e:
                env[e["name"]] = e["value"]
            elif (e.get("valueFrom") or {}).get("fieldRef", {}).get("fieldPath") == "spec.nodeName":
                env[e["name"]] = self.name
        probe = (c.get("readinessProbe") or {}).get("exec", {}).get("command")
        logs = self.host_root.parent / "pod-logs"
        logs.mkdir(parents=True, exist_ok=True)
        inits = []
        for ic in spec.get("initContainers") or []:
            cmd = self.init_images.get(ic.get("image", ""))
            inits.append({"name": ic["name"], "image": ic.get("image", ""),
                          "argv": list(cmd) + list(ic.get("args") or []) if cmd is not None else None})
        return _Container(pod=(ns, pname), daemonset=f"{ns}/{ref['name']}",
                          template=json.dumps(spec, sort_keys=True),
                          argv=self._agent_argv(list(c.get("command") or [])[1:] + list(c.get("args") or []), mounts),
                          probe=self._agent_argv(probe[1:], mounts) if probe else None, env=env,
                          grace_s=float(spec.get("terminationGracePeriodSeconds", 30)),
                          log_path=logs / f"{pname}.log", inits=inits, inits_done=not inits,
                          fallback_to_logs=c.get("terminationMessagePolicy") == "FallbackToLogsOnError")

    def _env(self, c: _Container) -> Dict[str, str]:
        env = dict(os.environ, **self.extra_env, **c.env)
        if self.sysfs_root is not None:
            env["SYSFS_ROOT"] = str(self.sysfs_root)
        return env

    async def _run_inits(self, c: _Container) -> bool:
        """Init containers in order, each to completion; False when one fails (retried later)."""
        for ic in c.inits:
            t = time.monotonic()
            if ic["argv"] is None:
                rc = -1  # ErrImagePull: no command for this image
            else:
                with open(c.log_path, "ab") as f:
                    p = await asyncio.create_subprocess_exec(*ic["argv"], env=self._env(c), stdout=f, stderr=f,
                                                             preexec_fn=self.netns.enter if self.netns else None)
                    rc = await p.wait()
            self.init_runs.append({"pod": c.pod[1], "name": ic["name"], "image": ic["image"], "rc": rc,
                                   "t_start": t, "t_end": time.monotonic()})
            if rc != 0:
                return False
        return True

    def _start(self, c: _Container) -> None:
        env = self._env(c)
        with open(c.log_path, "ab") as f:
            c.log_start = f.tell()
            c.proc = subprocess.Popen(c.argv, env=env, stdout=f, stderr=subprocess.STDOUT,
                                      preexec_fn=self.netns.enter if self.netns else None)
        c.started_at.append(time.monotonic())
        log.info("node %s: started %s (pid %d)", self.name, c.pod[1], c.proc.pid)

    async def _terminate(self, c: _Container) -> None:
        p = c.proc
        if p is None or p.poll() is not None:
            return
        t = time.monotonic()
        p.send_signal(signal.SIGTERM)
        end = t + c.grace_s
        while p.poll() is None and time.monotonic() < end:
            await asyncio.sleep(0.001)
        if p.poll() is None:
            p.kill()
            p.wait()
        self._record_exit(c, time.monotonic() - t)

    def _record_exit(self, c: _Container, sigterm_to_exit_s: Optional[float] = None) -> None:
        try:
            text = c.log_path.read_text(errors="replace")[-4000:]
        except OSError:
            text = ""
        self.exited.append({"pod": c.pod[1], "rc": c.proc.returncode if c.proc else None, "log": text,
                            "sigterm_to_exit_s": sigterm_to_exit_s})

    def _set_ready(self, c: _Container, ready: bool) -> None:
        if c.ready != ready:
            c.ready = ready
            self.fake.set_agent_ready(self.name, ready, daemonset=c.daemonset)

    def _terminated(self, c: _Container) -> dict:
        """``lastState.terminated`` as the kubelet records it: the exit code (128 + signal for a
        killed process) and, under FallbackToLogsOnError after a failure, the log tail of this
        run (at most 80 lines and 2048 bytes, whichever is smaller)."""
        rc = c.proc.returncode if c.proc else 0
        code = 128 - rc if rc < 0 else rc
        out = {"exitCode": code, "reason": "Completed" if code == 0 else "Error"}
        if code != 0 and c.fallback_to_logs:
            try:
                with open(c.log_path, "rb") as f:
                    f.seek(c.log_start)
                    tail = f.read()[-2048:]
            except OSError:
                tail = b""
            out["message"] = "\n".join(tail.decode(errors="replace").splitlines()[-80:])
        return out

    async def _kubelet(self) -> None:
        while not self._stop.is_set():
            pods = {(p["metadata"].get("namespace", ""), p["metadata"]["name"]): p
                    for p in self.fake.list_objects(kube.PODS) if (p.get("spec") or {}).get("nodeName") == self.name}
            for key in list(self.containers):
                if key not in pods:  # Pod deleted (DaemonSet gone or node deselected)
                    await self._terminate(self.containers[key])
                    del self.containers[key]
            for key, pod in pods.items():
                want = self._spec_for(pod)
                if want is None:
                    continue
                c = self.containers.get(key)
                if c is not None and c.template != want.template:  # rolling update of this node
                    self._set_ready(c, False)
                    await self._terminate(c)
                    c = None
                if c is None:
                    self.containers[key] = c = want
                if not c.inits_done:  # Init: the driver container before the agent
                    if time.monotonic() < c.next_start:
                        continue
                    if await self._run_inits(c):
                        c.inits_done, c.next_start = True, 0.0
                    else:  # Init:CrashLoopBackOff
                        c.next_start = time.monotonic() + c.backoff
                        c.backoff = min(c.backoff * 2, 5.0)
                        continue
                if c.proc is None:
                    self._start(c)
                elif c.proc.poll() is not None:  # crashed: restartPolicy Always
                    if c.next_start == 0.0:
                        self._record_exit(c)
                        c.ready = False
                        self.fake.set_agent_ready(self.name, False, daemonset=c.daemonset, terminated=self._terminated(c))
                        c.next_start = time.monotonic() + c.backoff
                        c.backoff = min(c.backoff * 2, 5.0)
                    elif time.monotonic() >= c.next_start:
                        c.next_start = 0.0
                        c.restarts += 1
                        self._start(c)
            await asyncio.sleep(0.005)

    async def _run_job(self, job: dict) -> None:
        ns, name = job["metadata"].get("namespace", ""), job["metadata"]["name"]
        spec = job["spec"]["template"]["spec"]
        c = spec["containers"][0]
        mounts = self._mounts(spec, c, name)
        for _, hp in mounts:
            self.host_path(hp).mkdir(parents=True, exist_ok=True)
        cmd = self.job_images.get(c.get("image", ""))
        cleanup = (job["metadata"].get("labels") or {}).get("app") == CLEANUP_APP
        if cleanup:  # the agent image, run as the node's agent binary (like the DaemonSet's Pods)
            cmd = []
            # The fake API server removes a deleted Pod at once; a real one keeps it until the
            # kubelet has stopped its containers, so the operator's "no agent Pods left" means the
            # agents have exited.  Keep that order here.
            ds = f"{ns}/{(job['metadata'].get('labels') or {}).get('amd.com/policy', '')}"
            while any(x.daemonset == ds and x.proc is not None and x.proc.poll() is None
                      for x in self.containers.values()):
                await asyncio.sleep(0.005)
        t = time.monotonic()
        rc = -1  # ErrImagePull: no command for this image
        if cmd is not None:
            if cleanup:
                argv = self._agent_argv(list(c.get("command") or [])[1:] + list(c.get("args") or []), mounts)
            else:
                argv = list(cmd) + [self._rewrite_arg(a, mounts) for a in c.get("args") or []]
            env = dict(os.environ, **self.extra_env, NODE_NAME=self.name)
            if self.sysfs_root is not None:
                env["SYSFS_ROOT"] = str(self.sysfs_root)
            logs = self.host_root.parent / "pod-logs"
            logs.mkdir(parents=True, exist_ok=True)
            with open(logs / f"{name}.log", "ab") as f:
                p = await asyncio.create_subprocess_exec(*argv, env=env, stdout=f, stderr=f,
                                                         preexec_fn=self.netns.enter if self.netns else None)
                rc = await p.wait()
        self.job_runs.append({"job": name, "rc": rc, "t_start": t, "t_end": time.monotonic()})
        if self.fake.get_object(kube.JOBS, name, ns) is not None:
            self.fake.set_job_result(name, ns, rc == 0)

    async def _jobs(self) -> None:
        while not self._stop.is_set():
            for job in self.fake.list_objects(kube.JOBS):
                spec = job["spec"]["template"]["spec"]
                uid = job["metadata"].get("uid")
                if spec.get("nodeName") != self.name or uid in self._jobs_started or job.get("status", {}).get(
                        "conditions"):
                    continue
                self._jobs_started.add(uid)
                self._tasks.append(asyncio.ensure_future(self._run_job(job)))
            await asyncio.sleep(0.01)

    async def _prober(self) -> None:
        while not self._stop.is_set():
            for c in list(self.containers.values()):
                if c.probe is None or c.proc is None or c.proc.poll() is not None:
                    continue
                probed = c.proc
                p = await asyncio.create_subprocess_exec(*c.probe, env=self._env(c), stdout=asyncio.subprocess.PIPE,
                                                         stderr=asyncio.subprocess.DEVNULL)
                out, _ = await p.communicate()
                rc = p.returncode
                # The kubelet drops a probe result of a container that has died meanwhile (its
                # exit already made the Pod unready): applying it would mark a dead agent ready.
                if c is self.containers.get(c.pod) and c.proc is probed and probed.poll() is None:
                    if rc != 0:  # the kubelet's event for a failed probe, with the probe's output
                        self.fake.record_probe_failure(c.pod[0], c.pod[1],
                                                       "Readiness probe failed: " + out.decode(errors="replace").strip())
                    self._set_ready(c, rc == 0)
            await asyncio.sleep(self.probe_period)

    # -- NFD worker --------------------------------------------------------------------------------
    def _read_features(self) -> Dict[str, str]:
        feats: Dict[str, str] = {}
        d = self.host_path(discovery.LABEL_FEATURES_DIR)
        try:
            names = sorted(os.listdir(d))
        except OSError:
            return feats
        for n in names:
            if n.startswith(".") or ".tmp" in n:
                continue
            try:
                text = (d / n).read_text()
            except OSError:
                continue
            for line in text.splitlines():
                line = line.strip()
                if not line or line.startswith("#"):
                    continue
                k, _, v = line.partition("=")
                feats[k.strip()] = v.strip() if _ else "true"
        return feats

    async def _nfd(self) -> None:
        while not self._stop.is_set():
            feats = self._read_features()
            if feats != self.features:
                self.features = feats
                self.fake.set_node_labels(self.name, dict(self.base_labels, **feats))
            await asyncio.sleep(self.nfd_period)

    # -- lifecycle ---------------------------------------------------------------------------------
    def node_labels(self) -> Dict[str, str]:
        n = self.fake.get_object(kube.NODES, self.name)
        return dict((n or {}).get("metadata", {}).get("labels") or {})

    async def start(self) -> None:
        if self.fake.get_object(kube.NODES, self.name) is None:
            self.fake.add_node(self.name, copy.deepcopy(self.base_labels))
        self._tasks = [asyncio.ensure_future(t()) for t in (self._kubelet, self._prober, self._nfd, self._jobs)]

    async def stop(self) -> None:
        """Node shutdown: every agent gets SIGTERM (and its grace period)."""
        self._stop.set()
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except asyncio.CancelledError:
                pass
        for key in list(self.containers):
            await self._terminate(self.containers.pop(key))
