# Reference Makefile:1-11 only builds an image; these targets build, test and bench.
PY ?= python3
TAG ?= $(shell git describe --tags --always --dirty 2>/dev/null || echo dev)
IMAGE ?= nanogpu/nano-gpu-scheduler-amd

.PHONY: native test test-gpu sanitize bench bench-configs image clean

native:
	$(PY) native/build.py

test: native
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu: native
	$(PY) -m pytest tests -q -m gpu

sanitize:
	$(PY) native/build.py --sanitize address
	$(PY) native/build.py --sanitize thread

bench: native
	$(PY) bench.py --steps 5 --warmup 1

bench-configs: native
	$(PY) -m nanogpu.sim.configs --out profiles/bench_configs.json

image:
	docker build -t $(IMAGE):$(TAG) .

clean:
	rm -rf native/build native/bin nanogpu/_native*.so nanogpu/_probe*.so
