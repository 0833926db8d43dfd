# MI355X (gfx950) training image.
# Counterpart of the reference image (reference: Dockerfile:1-49, which used
# tensorflow/tensorflow:latest-gpu + gcloud SDK + the kubernetes client).
# The HIP extensions are compiled for gfx950 at build time, in-tree.
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

ENV PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    TORCH_NCCL_ASYNC_ERROR_HANDLING=1 \
    PYTHONUNBUFFERED=1

WORKDIR /app
COPY pyproject.toml setup.py README.md /app/
COPY csrc /app/csrc
COPY tensorflow_distributed_on_gke_amd /app/tensorflow_distributed_on_gke_amd
COPY configuration /app/configuration
COPY __graft_entry__.py bench.py /app/

# PyYAML ships with the ROCm PyTorch image; google-cloud-storage is optional
# (storage_backend: gcs).
RUN python3 -c "from tensorflow_distributed_on_gke_amd import _build; _build.build(verbose=True)" && \
    pip install --no-deps -e .

# 3479: heartbeat / liveness HTTP, 3480: torch.distributed TCPStore rendezvous
# (the reference exposed 4793 but used 3479/3480, SURVEY.md §2.1 C33)
EXPOSE 3479 3480

CMD ["python3", "-u", "-m", "tensorflow_distributed_on_gke_amd", "train"]
