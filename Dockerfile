# Runtime image of the framework (replaces the reference's per-stage python:3.9-slim image,
# /root/reference/src/dockerfile:1, SURVEY R15): one image for every rank; the launcher starts
# one process per GPU inside it.
#   docker build -t dnn-amd .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --ipc=host \
#       dnn-amd python bench.py --gpus 1
#   docker run ... dnn-amd python -m torch.distributed.run --nproc-per-node 8 \
#       --master-addr 127.0.0.1 bench.py --gpus 8
# Base: any ROCm 7.x image with a ROCm build of PyTorch (torch's libamdhip64.so.7 is shared by
# the extension).
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

ENV HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTORCH_ROCM_ARCH=gfx950 \
    PYTHONUNBUFFERED=1
WORKDIR /opt/dnn
COPY . /opt/dnn
RUN python -m pip install --no-deps --no-build-isolation -e . && \
    python -m docker_dist_nn_amd._build
# stage ports keep the reference's scheme 5100 + 100*i + 1 (partition.py): 5101, 5201, ... 5801
EXPOSE 5101 5201 5301 5401 5501 5601 5701 5801
CMD ["python", "bench.py"]
