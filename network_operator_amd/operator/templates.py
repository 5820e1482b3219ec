"""The agent's workload as the reconciler builds it: the DaemonSet template's arguments, volumes,
probe, image and placement for each configurationType, and the constants the node-side contract
shares with the agent (artifact paths, label files).

Reference: updateGaudiScaleOutDaemonSet / addHostVolume (internal/controller/
networkconfiguration_controller.go:69-107,164-204): arguments fully recomputed from the spec in the
reference order, hostPath volumes DirectoryOrCreate in the reference order.  Fixes (SURVEY.md
§7.6): ``pullPolicy`` applied, volumes no longer wanted removed.  Pure functions on dicts; the
reconciler (reconciler.py) writes what they build.
"""

from __future__ import annotations

import copy
from typing import List, Optional

from .. import discovery
from ..api.v1alpha1 import types as T
from .holdoff import set_hold_off

ARTIFACT_DIR_HOST = "/etc/amd/scale-out"
ARTIFACT_DIR_CONTAINER = "/host" + ARTIFACT_DIR_HOST
RCCL_NET_FILE = "rccl-net.json"
RCCL_ENV_FILE = "rccl.env"
RCCL_TOPO_FILE = "rccl-topo.xml"
# --verify-peers: a switch answers ARP in well under a millisecond; 2 s covers a port that is
# still coming up, and stays far below the kubelet's restart back-off.
VERIFY_PEERS_TIMEOUT = "2s"
FW_LLDP_STATE_FILE = "fw-lldp-state"  # --fw-lldp-state: firmware LLDP originals kept by --keep-config agents
LLDP_CACHE_FILE = "lldp-cache"  # --lldp-cache, beside the artifacts so it survives pod restarts
# --link-state: each NIC's up/down from before the first agent, so the agent restarted after a
# crash (or a --keep-config restart) and the cleanup Job put back what no agent in memory saw.
LINK_STATE_FILE = "link-state"
L3_WAIT = "90s"

# Volumes the reconciler manages (the template's nfd-features is never touched).
MANAGED_VOLUMES = ("var-run-dbus", "networkmanager", "rccl-artifacts")


def add_host_volume(ds: dict, name: str, host_path: str, container_path: str,
                    volume_type: str = "DirectoryOrCreate") -> None:
    spec = ds["spec"]["template"]["spec"]
    vols = spec.setdefault("volumes", [])
    if any(v.get("name") == name for v in vols):
        return
    vols.append({"name": name, "hostPath": {"path": host_path, "type": volume_type}})
    containers = spec.get("containers") or []
    if containers:
        containers[0].setdefault("volumeMounts", []).append({"name": name, "mountPath": container_path})


def remove_volume(ds: dict, name: str) -> None:
    spec = ds["spec"]["template"]["spec"]
    spec["volumes"] = [v for v in spec.get("volumes", []) if v.get("name") != name]
    for c in spec.get("containers") or []:
        if "volumeMounts" in c:
            c["volumeMounts"] = [m for m in c["volumeMounts"] if m.get("name") != name]


def order_managed_volumes(ds: dict) -> None:
    """Volumes (and the agent's mounts) in one canonical order: the template's own first, then
    NetworkManager, then artifacts, then the driver container's -- the order the reference
    produces from scratch (controller_test.go:170-179), kept stable however the spec evolves."""
    rank = {n: i for i, n in enumerate(MANAGED_VOLUMES + ("host-lib-modules",))}
    key = lambda x: (x.get("name") in rank, rank.get(x.get("name"), 0))  # noqa: E731 (stable sort)
    pod = ds["spec"]["template"]["spec"]
    if "volumes" in pod:
        pod["volumes"] = sorted(pod["volumes"], key=key)
    for c in pod.get("containers") or []:
        if "volumeMounts" in c:
            c["volumeMounts"] = sorted(c["volumeMounts"], key=key)


def agent_args(p: T.NetworkClusterPolicy) -> List[str]:
    so = p.spec.amdScaleOut
    args = ["--configure=true", "--keep-running", f"--mode={so.layer}"]
    if p.spec.logLevel > 0:
        args.append(f"--v={p.spec.logLevel}")
    if so.mtu > 0:
        args.append(f"--mtu={so.mtu}")
    if so.disableNetworkManager:
        args += ["--disable-networkmanager", "--nm-keyfile-dir=/etc/NetworkManager/conf.d"]
    if so.layer == "L3":
        args += [f"--wait={so.lldpWait or L3_WAIT}", f"--rccl-net={ARTIFACT_DIR_CONTAINER}/{RCCL_NET_FILE}",
                 f"--rccl-env={ARTIFACT_DIR_CONTAINER}/{RCCL_ENV_FILE}"]
    else:
        # MI355X: RCCL needs the HCA list and the link-local RoCE v2 GID in L2 as well (Gaudi's
        # firmware did not, so the reference passes nothing in L2).
        args.append(f"--rccl-env={ARTIFACT_DIR_CONTAINER}/{RCCL_ENV_FILE}")
        if so.carrierWait:
            args.append(f"--carrier-wait={so.carrierWait}")
    # NCCL_TOPO_FILE: written through the agent's mount, named in rccl.env by the host path jobs
    # mount (the reference's HCCL contract is gaudinet.json, controller.go:198-200).
    args += [f"--rccl-topo={ARTIFACT_DIR_CONTAINER}/{RCCL_TOPO_FILE}",
             f"--rccl-topo-env-path={ARTIFACT_DIR_HOST}/{RCCL_TOPO_FILE}"]
    # MI355X options.  xgmiCheck and requireRdma are on unless the policy turns them off (the
    # webhook and the CRD default them; a policy stored before they existed reads them as unset).
    if so.xgmiCheck is not False:
        args.append("--xgmi-expect=0")
    if so.requireRdma is not False:
        args.append("--require-rdma")
        if so.rdmaWait:
            args.append(f"--rdma-wait={so.rdmaWait}")
    if so.lldpAnnounce is False:
        args.append("--lldp-announce=false")
    if so.interfaces:
        args.append("--interfaces=" + ",".join(so.interfaces))
    if so.nicDrivers:
        args.append("--nic-drivers=" + ",".join(so.nicDrivers))
    if so.disableFirmwareLldp and so.layer == "L3":
        args.append("--disable-fw-lldp")
        if so.handDcbxToHost:  # opt-in: the NIC firmware stops negotiating PFC/ETS
            args.append("--fw-lldp-dcbx-host")
    if so.metricsPort:
        args.append(f"--metrics-bind-address=:{so.metricsPort}")
    if so.railTableBase and so.layer == "L3":
        args.append(f"--rail-table-base={so.railTableBase}")
    if so.rcclSocketIfname:
        args.append(f"--rccl-socket-ifname={so.rcclSocketIfname}")
    if (so.lldpCache or so.keepConfigOnRestart) and so.layer == "L3":
        # keepConfigOnRestart: the cache is what lets the next agent adopt the addresses it finds
        args.append(f"--lldp-cache={ARTIFACT_DIR_CONTAINER}/{LLDP_CACHE_FILE}")
    if so.keepConfigOnRestart:
        args.append("--keep-config")
    if so.disableFirmwareLldp and so.layer == "L3":
        # The originals of what --disable-fw-lldp changes, on the node: with --keep-config they stay
        # changed across restarts and the cleanup Job restores them; without, they outlive an agent
        # that fails and the next clean exit restores them.
        args.append(f"--fw-lldp-state={ARTIFACT_DIR_CONTAINER}/{FW_LLDP_STATE_FILE}")
    if so.railSwitchPattern and so.layer == "L3":
        args.append(f"--rail-switch-pattern={so.railSwitchPattern}")
    if so.minLinkSpeedGbps:
        args.append(f"--min-link-speed-gbps={so.minLinkSpeedGbps}")
    if so.requireFullPcieLink:
        args.append("--require-full-pcie")
    if so.allowPolicyRouted:
        args.append("--allow-policy-routed")
    if so.checkPeerMtu is False and so.layer == "L3":
        args.append("--check-peer-mtu=false")
    args.append(f"--link-state={ARTIFACT_DIR_CONTAINER}/{LINK_STATE_FILE}")
    args.append(f"--status-file={discovery.AGENT_STATUS_FILE}")
    if so.verifyPeers and so.layer == "L3":
        args.append(f"--verify-peers={VERIFY_PEERS_TIMEOUT}")
    if so.rcclEnv:
        args.append("--rccl-env-extra=" + ",".join(f"{k}={v}" for k, v in sorted(so.rcclEnv.items())))
    if so.gpuDirectRdma:
        args.append("--require-gdr=" + {"Any": "any", "PeerMem": "peermem", "DmaBuf": "dmabuf"}[so.gpuDirectRdma])
    return args


def update_amd_scale_out_daemonset(ds: dict, p: T.NetworkClusterPolicy, namespace: str) -> None:
    """updateGaudiScaleOutDaemonSet (:164-204) for amd-so."""
    md = ds.setdefault("metadata", {})
    md["name"] = p.name
    md["namespace"] = namespace
    pod = ds["spec"]["template"]["spec"]
    if p.spec.nodeSelector:
        pod["nodeSelector"] = dict(p.spec.nodeSelector)
    c = pod["containers"][0]
    so = p.spec.amdScaleOut
    if so.image:
        c["image"] = so.image
    if so.pullPolicy:
        c["imagePullPolicy"] = so.pullPolicy
    wanted = set()
    if so.disableNetworkManager:
        add_host_volume(ds, "var-run-dbus", "/var/run/dbus", "/var/run/dbus")
        add_host_volume(ds, "networkmanager", "/etc/NetworkManager", "/etc/NetworkManager")
        wanted |= {"var-run-dbus", "networkmanager"}
    add_host_volume(ds, "rccl-artifacts", ARTIFACT_DIR_HOST, ARTIFACT_DIR_CONTAINER)  # L2 too (rccl.env)
    wanted.add("rccl-artifacts")
    # The rails' RDMA driver (KMD) container, as for host-nic: the RDMA devices exist when the
    # agent starts, and --require-rdma finds them without waiting.
    if set_driver_container(pod, so.driverImage, so.pullPolicy):
        wanted.add("host-lib-modules")
    for v in MANAGED_VOLUMES + ("host-lib-modules",):
        if v not in wanted:
            remove_volume(ds, v)
    order_managed_volumes(ds)
    probe = c.get("readinessProbe", {}).get("exec")
    if probe:
        probe["command"] = probe["command"][:1] + ["--ready-check", f"--status-file={discovery.AGENT_STATUS_FILE}"]
    # Agent metrics port (hostNetwork: the container port is the node port).
    ports = [x for x in c.get("ports", []) if x.get("name") != "metrics"]
    if so.metricsPort:
        ports.append({"name": "metrics", "containerPort": so.metricsPort, "protocol": "TCP"})
    if ports:
        c["ports"] = ports
    else:
        c.pop("ports", None)
    c["args"] = agent_args(p)


HOST_NIC_LABEL = "amd.feature.node.kubernetes.io/host-nic-ready"
HOST_NIC_LABEL_FILE = "host-nic-readiness.txt"
HOST_NIC_LLDP_CACHE_FILE = "host-nic-lldp-cache"
HOST_NIC_MTU_STATE_FILE = "host-nic-mtu-state"  # --mtu-state: the host NICs' own MTUs
HOST_NIC_LINK_STATE_FILE = "host-nic-link-state"  # --link-state, apart from the amd-so agent's
DRIVER_CONTAINER = "nic-driver"


def set_driver_container(pod: dict, image: str, pull_policy: str) -> bool:
    """The optional kernel-driver (KMD) init container: privileged, sees the host's modules, runs
    to completion before the agent starts, so the NICs (host-nic) or their RDMA devices (amd-so)
    exist when discovery runs.  Removed when `image` is empty; True when it is there."""
    inits = [x for x in pod.get("initContainers", []) if x.get("name") != DRIVER_CONTAINER]
    if image:
        spec_vols = pod.setdefault("volumes", [])
        if not any(v.get("name") == "host-lib-modules" for v in spec_vols):
            spec_vols.append({"name": "host-lib-modules", "hostPath": {"path": "/lib/modules", "type": "Directory"}})
        inits.append({"name": DRIVER_CONTAINER, "image": image, "imagePullPolicy": pull_policy or "IfNotPresent",
                      "securityContext": {"privileged": True},
                      "volumeMounts": [{"name": "host-lib-modules", "mountPath": "/lib/modules"}]})
    if inits:
        pod["initContainers"] = inits
    else:
        pod.pop("initContainers", None)
    return bool(image)


def host_nic_agent_args(p: T.NetworkClusterPolicy) -> List[str]:
    """Agent flags for ``host-nic``: RDMA NIC discovery instead of GPU affinity, its own readiness
    label and file (so it can coexist with an ``amd-so`` policy on the same node)."""
    hn = p.spec.hostNic or T.HostNicSpec()
    args = ["--configure=true", "--keep-running", f"--mode={hn.layer}",
            "--nic-discovery=" + ("none" if hn.interfaces else "rdma"),
            f"--nfd-label-file={HOST_NIC_LABEL_FILE}", f"--nfd-label={HOST_NIC_LABEL}"]
    if p.spec.logLevel > 0:
        args.append(f"--v={p.spec.logLevel}")
    if hn.mtu > 0:
        args.append(f"--mtu={hn.mtu}")
    # The node's own NICs get their MTU back when the agent goes for good: on a clean exit, or
    # (keepConfigOnRestart) from the record the cleanup Job reads.  Always, not only while mtu is
    # set: the agent applies its default MTU otherwise, and a policy that dropped mtu must still
    # let the next agent and the cleanup Job find and restore the record.
    args += ["--restore-mtu", f"--mtu-state={ARTIFACT_DIR_CONTAINER}/{HOST_NIC_MTU_STATE_FILE}"]
    if hn.disableNetworkManager:
        args += ["--disable-networkmanager", "--nm-keyfile-dir=/etc/NetworkManager/conf.d"]
    if hn.layer == "L3":
        args.append(f"--wait={hn.lldpWait or L3_WAIT}")
        if hn.verifyPeers:
            args.append(f"--verify-peers={VERIFY_PEERS_TIMEOUT}")
    elif hn.carrierWait:
        args.append(f"--carrier-wait={hn.carrierWait}")
    if hn.interfaces:
        args.append("--interfaces=" + ",".join(hn.interfaces))
    if hn.nicDrivers:
        args.append("--nic-drivers=" + ",".join(hn.nicDrivers))
    if hn.includeGpuRails and not hn.interfaces:
        args.append("--rdma-include-gpu-rails")
    if hn.checkPeerMtu is False and hn.layer == "L3":
        args.append("--check-peer-mtu=false")
    if hn.minLinkSpeedGbps:
        args.append(f"--min-link-speed-gbps={hn.minLinkSpeedGbps}")
    if hn.requireFullPcieLink:
        args.append("--require-full-pcie")
    if hn.allowPolicyRouted:
        args.append("--allow-policy-routed")
    if hn.keepConfigOnRestart:
        if hn.layer == "L3":  # its own cache beside the scale-out agent's
            args.append(f"--lldp-cache={ARTIFACT_DIR_CONTAINER}/{HOST_NIC_LLDP_CACHE_FILE}")
        args.append("--keep-config")
    args += [f"--link-state={ARTIFACT_DIR_CONTAINER}/{HOST_NIC_LINK_STATE_FILE}",
             f"--status-file={discovery.AGENT_STATUS_FILE}"]
    return args


def update_host_nic_daemonset(ds: dict, p: T.NetworkClusterPolicy, namespace: str) -> None:
    """The ``host-nic`` branch (the reference's "Future work": Host-NIC use + KMD install)."""
    hn = p.spec.hostNic or T.HostNicSpec()
    md = ds.setdefault("metadata", {})
    md["name"] = p.name
    md["namespace"] = namespace
    pod = ds["spec"]["template"]["spec"]
    if p.spec.nodeSelector:
        pod["nodeSelector"] = dict(p.spec.nodeSelector)
    c = pod["containers"][0]
    if hn.image:
        c["image"] = hn.image
    if hn.pullPolicy:
        c["imagePullPolicy"] = hn.pullPolicy
    wanted = set()
    if hn.disableNetworkManager:
        add_host_volume(ds, "var-run-dbus", "/var/run/dbus", "/var/run/dbus")
        add_host_volume(ds, "networkmanager", "/etc/NetworkManager", "/etc/NetworkManager")
        wanted |= {"var-run-dbus", "networkmanager"}
    # The MTU and link-state records (and the L3 LLDP cache) outlive the Pod: always mounted, so a
    # policy that dropped mtu still lets the next agent and the cleanup Job find the record.
    add_host_volume(ds, "rccl-artifacts", ARTIFACT_DIR_HOST, ARTIFACT_DIR_CONTAINER)
    wanted.add("rccl-artifacts")
    if set_driver_container(pod, hn.driverImage, hn.pullPolicy):
        wanted.add("host-lib-modules")
    for v in MANAGED_VOLUMES + ("host-lib-modules",):
        if v not in wanted:
            remove_volume(ds, v)
    order_managed_volumes(ds)
    probe = c.get("readinessProbe", {}).get("exec")
    if probe:
        probe["command"] = [probe["command"][0], "--ready-check", f"--nfd-label-file={HOST_NIC_LABEL_FILE}",
                            f"--status-file={discovery.AGENT_STATUS_FILE}"]
    c["args"] = host_nic_agent_args(p)


def update_daemonset_for(ds: dict, p: T.NetworkClusterPolicy, namespace: str,
                         hold_off: Optional[List[dict]] = None) -> None:
    """createDaemonSet / updateDaemonSet dispatch on configurationType (:243-265).  Also the
    rolling-update width (spec.maxUnavailable; 1 when unset, like the reference's DaemonSet) and
    the node affinity that holds the agents off nodes an older policy of the type selects."""
    ds["spec"].setdefault("updateStrategy", {"type": "RollingUpdate"}).setdefault("rollingUpdate", {})[
        "maxUnavailable"] = p.spec.maxUnavailable if p.spec.maxUnavailable is not None else 1
    if p.spec.configurationType == T.CONFIG_AMD_SCALE_OUT:
        update_amd_scale_out_daemonset(ds, p, namespace)
    elif p.spec.configurationType == T.CONFIG_HOST_NIC:
        update_host_nic_daemonset(ds, p, namespace)
    else:
        raise ValueError(f"unknown configuration type {p.spec.configurationType!r}")
    # Tainted GPU nodes (amd.com/gpu:NoSchedule, ...): the policy's tolerations, exactly (a
    # toleration removed from the policy leaves the template; the cleanup Job copies this spec).
    pod = ds["spec"]["template"]["spec"]
    if p.spec.tolerations:
        pod["tolerations"] = copy.deepcopy(p.spec.tolerations)
    else:
        pod.pop("tolerations", None)
    if p.spec.priorityClassName:
        pod["priorityClassName"] = p.spec.priorityClassName
    else:
        pod.pop("priorityClassName", None)
    set_hold_off(pod, hold_off)
