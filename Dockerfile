# Engine / gateway / exporter image for MI355X (gfx950).  Built on the node by
# provision/llm-d-deploy.yaml (podman -> CRI-O shared storage, no registry needed).
#
# The stack is pinned to the one every test, bench and the in-tree extension ABI ran on:
# ROCm 7.2 userspace + torch 2.10.0+rocm7.0 (tests/test_provisioning.py checks
# TORCH_VERSION against the torch the build compiles _C.so against, and the image
# build asserts it again after installing).  _C.so links libtorch directly and the MoE
# prefill uses torch._grouped_mm, so a different torch is a different product.
ARG ROCM_BASE=docker.io/rocm/dev-ubuntu-22.04:7.2-complete
ARG TORCH_VERSION=2.10.0+rocm7.0
ARG TORCH_INDEX=https://download.pytorch.org/whl/rocm7.0
FROM ${ROCM_BASE}
ARG TORCH_VERSION
ARG TORCH_INDEX
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
RUN apt-get update && apt-get install -y --no-install-recommends python3-pip python3-dev g++ \
    && rm -rf /var/lib/apt/lists/*
RUN pip install --no-cache-dir "torch==${TORCH_VERSION}" --index-url "${TORCH_INDEX}" \
    && pip install --no-cache-dir fastapi uvicorn aiohttp jinja2 pyyaml safetensors pybind11 \
       numpy prometheus_client \
    && python3 -c "import torch, sys; v = torch.__version__; \
sys.exit(0 if v == '${TORCH_VERSION}' else 'torch ' + v + ' != pinned ${TORCH_VERSION}')"
WORKDIR /opt/akap
COPY . /opt/akap
# compile the gfx950 HIP kernels + the C++ runtime in-tree (content-addressed: the source
# digest is compiled into _C.so and checked at load time)
RUN python3 -m aws_k8s_ansible_provisioner_amd.build_ext -j 16
ENV PYTHONPATH=/opt/akap
EXPOSE 8000 8080 9400
ENTRYPOINT []
CMD ["python3", "-m", "aws_k8s_ansible_provisioner_amd.server"]
