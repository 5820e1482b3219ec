# AMD MI355X network operator — developer targets.
PYTHON ?= python3
JOBS   ?= 8
IMG_OPERATOR ?= amd/amd-network-operator:0.1.0
IMG_AGENT    ?= amd/amd-network-linkdiscovery:0.1.0
IMG_VALIDATION ?= amd/amd-network-validation:0.1.0
IMG_RDMA_DRIVER ?= amd/amd-network-rdma-driver:0.1.0

KUBECTL ?= kubectl
CONTAINER_TOOL ?= docker
HELM ?= helm
RELEASE_REGISTRY ?= ghcr.io/amd/network-operator
# MI355X hosts are x86-64; the operator image is pure Python and builds for arm64 too.
PLATFORMS ?= linux/amd64
VERSION ?= 0.1.0
BUNDLE_IMG ?= amd/amd-network-operator-bundle:v$(VERSION)

.PHONY: all help build native hip test test-native test-netns test-gpu manifests deployments bench bench-node-ready bench-e2e \
        images sanitize tsan clean fmt vet lint fuzz run build-installer install uninstall deploy undeploy bundle \
        bundle-build helm-package-chart fuzz-native check-hardening catalog-build catalog-push bundle-push \
        generate test-e2e lint-fix operator-image operator-push discover-image discover-push validation-image \
        validation-push rdma-driver-image rdma-driver-push docker-buildx helm-update-dependencies helm-push-chart

all: build

help:                       ## list targets
	@grep -E '^[a-zA-Z_-]+:.*## ' $(MAKEFILE_LIST) | awk -F':.*## ' '{printf "  %-20s %s\n", $$1, $$2}'

build:                      ## C++ agent + pybind module + HIP (gfx950) library, in-tree
	$(PYTHON) -c 'import __graft_entry__ as g; g.build()'

native:
	cmake -S native -B _build -G Ninja && cmake --build _build -j$(JOBS)

hip:
	$(MAKE) -C native/hip ARCH=gfx950 -j$(JOBS)

test:                       ## everything that runs without a GPU
	$(PYTHON) -m pytest tests -q -m "not gpu"

test-e2e:                   ## end-to-end: operator + simulated kubelet/NFD + real agent in network namespaces
	$(PYTHON) -m pytest tests/test_e2e.py tests/test_helm_install.py -v

test-native:
	network_operator_amd/_lib/bin/netop-unit-tests

check-hardening:            ## PIE / full RELRO / NX stack / stack protector / FORTIFY on the agent binaries (checksec gate)
	$(PYTHON) tools/check_hardening.py network_operator_amd/_lib/bin/discover network_operator_amd/_lib/bin/netop-topo network_operator_amd/_lib/bin/netop-lldp-tx

test-netns:                 ## veth + synthetic-switch integration and the end-to-end runs (root or user namespaces)
	$(PYTHON) -m pytest tests/test_netns_integration.py tests/test_e2e.py -q

test-gpu:                   ## on an MI355X box
	$(PYTHON) -m pytest tests -q -m gpu

test-netns-asan: sanitize   ## the veth + synthetic-switch scenarios against the ASan+UBSan agent
	NETOP_BIN_DIR=$(CURDIR)/_build-asan/out/bin ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 \
	  $(PYTHON) -m pytest tests/test_netns_integration.py tests/test_e2e.py -q

sanitize:                   ## host-side ASan+UBSan build of the agent and its unit suite
	cmake -S native -B _build-asan -G Ninja -DNETOP_SANITIZE=ON -DNETOP_PYTHON=OFF -DNETOP_OUT=$(CURDIR)/_build-asan/out && \
	cmake --build _build-asan -j$(JOBS) && _build-asan/out/bin/netop-unit-tests

tsan:                       ## ThreadSanitizer build of the agent and its unit suite (metrics thread)
	cmake -S native -B _build-tsan -G Ninja -DNETOP_TSAN=ON -DNETOP_PYTHON=OFF -DNETOP_OUT=$(CURDIR)/_build-tsan/out && \
	cmake --build _build-tsan -j$(JOBS) && TSAN_OPTIONS=halt_on_error=1 _build-tsan/out/bin/netop-unit-tests

manifests:                  ## regenerate the CRD and every generated kustomize / Helm manifest
	$(PYTHON) -m network_operator_amd.api.v1alpha1.crd
	$(PYTHON) -m network_operator_amd.packaging.manifests

generate: manifests         ## alias: the CRD, webhook and RBAC manifests are generated from the Python types (no deepcopy codegen: copy.deepcopy)

deployments:                ## render kustomize + Helm offline into deployments/
	mkdir -p deployments
	$(PYTHON) -c 'from network_operator_amd.testing.render import *; open("deployments/operator.yaml","w").write(dump_all(kustomize_build("config/operator/default")))'
	$(PYTHON) -c 'from network_operator_amd.testing.render import *; open("deployments/helm-default.yaml","w").write(dump_all(helm_template("charts/network-operator", {"config":{"amd":{"enabled":True}}}, "amd-network-operator")))'
	$(PYTHON) -m network_operator_amd.testing.render --discovery config/operator/samples/amd-l3.yaml > deployments/discovery.yaml
	$(PYTHON) -m network_operator_amd.testing.render --discovery config/operator/samples/amd-host-nic.yaml > deployments/discovery-host-nic.yaml

bench:                      ## 1-GPU RCCL bench (driver contract); N GPUs: torchrun --nproc-per-node N bench.py --gpus N
	$(PYTHON) bench.py --gpus 1 --steps 20 --warmup 5

bench-node-ready:           ## node scale-out-ready latency in the netns harness
	$(PYTHON) bench/node_ready.py --nics 8 --runs 5

bench-e2e:                  ## policy created -> Node labelled / status All good (operator + simulated node + agent)
	$(PYTHON) bench/node_ready.py --e2e --nics 8 --runs 20

fmt:                        ## clang-format the native sources (if installed)
	@command -v clang-format >/dev/null && clang-format -i native/src/*.cpp native/include/netop/*.hpp native/tests/*.cpp native/tools/*.cpp || echo "clang-format not installed"

vet:                        ## byte-compile and check Python (tools/pycheck.py), warnings-as-errors C++ build of the agent
	$(PYTHON) -m compileall -q network_operator_amd bench bench.py __graft_entry__.py
	$(PYTHON) tools/pycheck.py
	cmake -S native -B _build-vet -G Ninja -DNETOP_PYTHON=OFF -DCMAKE_CXX_FLAGS=-Werror -DNETOP_OUT=$(CURDIR)/_build-vet/out && \
	cmake --build _build-vet -j$(JOBS)

lint: vet                   ## vet + drift checks (CRD, generated manifests, rendered deployments)
	$(PYTHON) -m network_operator_amd.packaging.manifests --check
	$(PYTHON) -m pytest tests/test_packaging.py -q

lint-fix: fmt manifests deployments  ## rewrite what lint checks: formatting, generated manifests, rendered deployments

fuzz:                       ## property-based CR churn + LLDP / Port Description fuzzing
	$(PYTHON) -m pytest tests/test_fuzz.py tests/test_native.py -q -k "fuzz or property or garbage or churn"

run:                        ## run the operator against the current kubeconfig (webhooks off)
	ENABLE_WEBHOOKS=false $(PYTHON) -m network_operator_amd.operator --health-probe-bind-address=:8081

build-installer:            ## dist/install.yaml: CRD + RBAC + webhooks + Deployment in one file
	$(PYTHON) -m network_operator_amd.packaging installer --out dist/install.yaml $(if $(IMG),--img $(IMG))

install: manifests          ## install the CRD into the current cluster
	$(KUBECTL) apply -f config/operator/crd/bases/amd.com_networkclusterpolicies.yaml

uninstall:                  ## remove the CRD from the current cluster
	$(KUBECTL) delete --ignore-not-found -f config/operator/crd/bases/amd.com_networkclusterpolicies.yaml

deploy: build-installer     ## deploy the operator into the current cluster
	$(KUBECTL) apply -f dist/install.yaml

undeploy:                   ## remove the operator from the current cluster
	$(KUBECTL) delete --ignore-not-found -f dist/install.yaml

bundle:                     ## OLM bundle (bundle/manifests, bundle/metadata, bundle.Dockerfile)
	$(PYTHON) -m network_operator_amd.packaging bundle --out bundle --version $(VERSION) --img $(IMG_OPERATOR)

bundle-build: bundle        ## build the OLM bundle image
	docker build -f bundle.Dockerfile -t $(BUNDLE_IMG) .

bundle-push:                ## push the OLM bundle image
	docker push $(BUNDLE_IMG)

# OLM catalog (file-based catalog index) from the bundle image(s); needs `opm` on PATH
# (the reference downloads it, Makefile:300-335; there is no network here, so bring your own).
OPM ?= opm
CATALOG_IMG ?= amd/amd-network-operator-catalog:v$(VERSION)
BUNDLE_IMGS ?= $(BUNDLE_IMG)
ifneq ($(origin CATALOG_BASE_IMG), undefined)
FROM_INDEX_OPT := --from-index $(CATALOG_BASE_IMG)
endif

catalog-build:              ## build a catalog image containing $(BUNDLE_IMGS) (opm index add)
	$(OPM) index add --container-tool docker --mode semver --tag $(CATALOG_IMG) --bundles $(BUNDLE_IMGS) $(FROM_INDEX_OPT)

catalog-push:               ## push the catalog image
	docker push $(CATALOG_IMG)

helm-update-dependencies:   ## fetch the NFD subchart (needs helm and the network)
	$(HELM) dependency update charts/network-operator

helm-package-chart:         ## .charts/<chart>-<version>.tgz
	$(PYTHON) -m network_operator_amd.packaging helm --out .charts

helm-push-chart: helm-package-chart  ## push the packaged chart to oci://$(RELEASE_REGISTRY)
	for c in .charts/*.tgz; do $(HELM) push $$c oci://$(RELEASE_REGISTRY) || exit 1; done

images: operator-image discover-image validation-image  ## all three images

operator-image:             ## control-plane image (distroless, nonroot)
	$(CONTAINER_TOOL) build -f build/Dockerfile.operator -t $(IMG_OPERATOR) .

operator-push:
	$(CONTAINER_TOOL) push $(IMG_OPERATOR)

discover-image:             ## node agent image (unit suite + hardening gate run in the build)
	$(CONTAINER_TOOL) build -f build/Dockerfile.linkdiscovery -t $(IMG_AGENT) .

discover-push:
	$(CONTAINER_TOOL) push $(IMG_AGENT)

validation-image:           ## fabric validation Job image (RCCL + HIP, gfx950)
	$(CONTAINER_TOOL) build -f build/Dockerfile.validation -t $(IMG_VALIDATION) .

validation-push:
	$(CONTAINER_TOOL) push $(IMG_VALIDATION)

rdma-driver-image:          ## RDMA driver init container (driverImage): modprobe of the NICs' RDMA drivers
	$(CONTAINER_TOOL) build -f build/Dockerfile.rdma-driver -t $(IMG_RDMA_DRIVER) .

rdma-driver-push:
	$(CONTAINER_TOOL) push $(IMG_RDMA_DRIVER)

# Multi-platform build and push of the operator image.  The Dockerfile already names its
# stages' bases, so buildx only needs --platform; a throwaway builder keeps the host's default.
docker-buildx:              ## build and push the operator image for $(PLATFORMS)
	- $(CONTAINER_TOOL) buildx create --name amd-netop-builder
	$(CONTAINER_TOOL) buildx use amd-netop-builder
	- $(CONTAINER_TOOL) buildx build --push --platform=$(PLATFORMS) --tag $(IMG_OPERATOR) -f build/Dockerfile.operator .
	- $(CONTAINER_TOOL) buildx rm amd-netop-builder

clean:
	rm -rf _build _build-asan _build-vet network_operator_amd/_lib deployments dist bundle bundle.Dockerfile .charts

FUZZ_CXX ?= /opt/rocm/lib/llvm/bin/clang++
FUZZ_TIME ?= 60
fuzz-native:                ## libFuzzer (+ASan/UBSan) on the LLDP, D-Bus, Port Description / state records / gpu_metrics, netlink and ARP parsers
	mkdir -p _build-fuzz
	for t in 1:lldp 2:dbus 3:portdesc 4:netlink 5:arp; do id=$${t%%:*}; name=$${t##*:}; \
	  $(FUZZ_CXX) -std=c++17 -O1 -g -fsanitize=fuzzer,address,undefined -fno-sanitize-recover=undefined \
	    -mllvm -asan-globals=0 \
	    -DNETOP_FUZZ_TARGET=$$id -DNETOP_VERSION='"fuzz"' -Inative/include native/fuzz/fuzz_targets.cpp \
	    native/src/common.cpp native/src/log.cpp native/src/lldp.cpp native/src/l3.cpp native/src/netlink.cpp \
	    native/src/dbus.cpp native/src/arp.cpp native/src/ethtool.cpp native/src/artifacts.cpp native/src/topology.cpp native/src/bounded.cpp \
	    -o _build-fuzz/fuzz_$$name -lpthread || exit 1; \
	  mkdir -p _build-fuzz/corpus_$$name; \
	  if [ $$name = portdesc ]; then cp tests/fixtures/gpu_metrics_v1_8.bin _build-fuzz/corpus_$$name/; fi; \
	  _build-fuzz/fuzz_$$name native/fuzz/regressions/* > _build-fuzz/$$name.replay.log 2>&1 || { tail -20 _build-fuzz/$$name.replay.log; exit 1; }; \
	  _build-fuzz/fuzz_$$name -artifact_prefix=_build-fuzz/$$name- -max_total_time=$(FUZZ_TIME) -rss_limit_mb=2048 \
	    -print_final_stats=1 _build-fuzz/corpus_$$name > _build-fuzz/$$name.log 2>&1; rc=$$?; \
	  grep -E "stat::number_of_executed_units|SUMMARY|ERROR" _build-fuzz/$$name.log | sed "s/^/$$name: /"; \
	  [ $$rc -eq 0 ] || exit $$rc; \
	done
