# nano-gpu-scheduler for MI355X: extender + node agent in one image.
# Reference: Dockerfile:1-18 (golang:1.16 build, debian runtime). Here the native core is
# C++17 (g++) and the probe is HIP for gfx950 (hipcc), so the build stage is a ROCm image.
FROM rocm/dev-ubuntu-22.04:7.2 AS build
# libssl-dev: the native bind writers speak TLS to kube-apiserver (native/src/kubewriter.cpp)
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip g++ libssl-dev && \
    pip3 install --no-cache-dir pybind11 aiohttp pyyaml prometheus_client grpcio protobuf
WORKDIR /src
COPY native native
COPY nanogpu nanogpu
COPY __graft_entry__.py pyproject.toml ./
RUN python3 native/build.py --force

FROM rocm/dev-ubuntu-22.04:7.2
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip libssl3 && \
    pip3 install --no-cache-dir aiohttp pyyaml prometheus_client grpcio protobuf && rm -rf /var/lib/apt/lists/*
WORKDIR /app
COPY --from=build /src/nanogpu nanogpu
COPY --from=build /src/native/bin/nanogpu-topo /usr/local/bin/nanogpu-topo
ENV PYTHONUNBUFFERED=1 NANOGPU_AUTOBUILD=0
EXPOSE 39999
ENTRYPOINT ["python3", "-m", "nanogpu"]
