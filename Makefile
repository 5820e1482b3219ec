# AMD MI355X network operator — developer targets.
PYTHON ?= python3
JOBS   ?= 8
IMG_OPERATOR ?= amd/amd-network-operator:0.1.0
IMG_AGENT    ?= amd/amd-network-linkdiscovery:0.1.0

.PHONY: all build native hip test test-native test-netns test-gpu manifests deployments bench bench-node-ready \
        images sanitize clean

all: build

build:                      ## C++ agent + pybind module + HIP (gfx950) library, in-tree
	$(PYTHON) -c 'import __graft_entry__ as g; g.build()'

native:
	cmake -S native -B _build -G Ninja && cmake --build _build -j$(JOBS)

hip:
	$(MAKE) -C native/hip ARCH=gfx950 -j$(JOBS)

test:                       ## everything that runs without a GPU
	$(PYTHON) -m pytest tests -q -m "not gpu"

test-native:
	network_operator_amd/_lib/bin/netop-unit-tests

test-netns:                 ## veth + synthetic-switch integration (root or user namespaces)
	$(PYTHON) -m pytest tests/test_netns_integration.py -q

test-gpu:                   ## on an MI355X box
	$(PYTHON) -m pytest tests -q -m gpu

sanitize:                   ## host-side ASan+UBSan build of the agent and its unit suite
	cmake -S native -B _build-asan -G Ninja -DNETOP_SANITIZE=ON -DNETOP_PYTHON=OFF -DNETOP_OUT=$(CURDIR)/_build-asan/out && \
	cmake --build _build-asan -j$(JOBS) && _build-asan/out/bin/netop-unit-tests

manifests:                  ## regenerate the CRD (kustomize base + Helm chart copy)
	$(PYTHON) -m network_operator_amd.api.v1alpha1.crd

deployments:                ## render kustomize + Helm offline into deployments/
	mkdir -p deployments
	$(PYTHON) -c 'from network_operator_amd.testing.render import *; open("deployments/operator.yaml","w").write(dump_all(kustomize_build("config/operator/default")))'
	$(PYTHON) -c 'from network_operator_amd.testing.render import *; open("deployments/helm-default.yaml","w").write(dump_all(helm_template("charts/network-operator", {"config":{"amd":{"enabled":True}}}, "amd-network-operator")))'

bench:                      ## 1-GPU RCCL bench (driver contract); N GPUs: torchrun --nproc-per-node N bench.py --gpus N
	$(PYTHON) bench.py --gpus 1 --steps 20 --warmup 5

bench-node-ready:           ## node scale-out-ready latency in the netns harness
	$(PYTHON) bench/node_ready.py --nics 8 --runs 5

images:
	docker build -f build/Dockerfile.operator -t $(IMG_OPERATOR) .
	docker build -f build/Dockerfile.linkdiscovery -t $(IMG_AGENT) .

clean:
	rm -rf _build _build-asan network_operator_amd/_lib deployments
