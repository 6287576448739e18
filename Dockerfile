# Engine / gateway / exporter image for MI355X (gfx950).  Built on the node by
# provision/llm-d-deploy.yaml (podman -> CRI-O shared storage, no registry needed).
# Base: ROCm 7.x + PyTorch-ROCm (the same stack this repo is developed against).
ARG BASE=docker.io/rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.8.0
FROM ${BASE}
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
RUN pip install --no-cache-dir fastapi uvicorn aiohttp jinja2 pyyaml safetensors pybind11
WORKDIR /opt/akap
COPY . /opt/akap
# compile the gfx950 HIP kernels + the C++ runtime in-tree
RUN python3 -m aws_k8s_ansible_provisioner_amd.build_ext -j 16
ENV PYTHONPATH=/opt/akap
EXPOSE 8000 8080 9400
ENTRYPOINT []
CMD ["python3", "-m", "aws_k8s_ansible_provisioner_amd.server"]
