# V-Gate on MI355X (gfx950). Two targets:
#   docker build --target rocm -t vgate:0.3.2-rocm .   # GPU image, native HIP engine
#   docker build --target cpu  -t vgate:0.3.2-cpu  .   # gateway / dry-run image, no GPU stack
# Run the GPU image with the ROCm device nodes:
#   docker run --device /dev/kfd --device /dev/dri --group-add video --group-add render \
#     --security-opt seccomp=unconfined --shm-size 16g -p 8000:8000 vgate:0.3.2-rocm

ARG ROCM_IMAGE=rocm/pytorch:rocm7.2_ubuntu22.04_py3.10_pytorch_release_2.10.0

FROM ${ROCM_IMAGE} AS rocm
ENV PYTHONUNBUFFERED=1 \
    PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    VGATE_DRY_RUN=false
WORKDIR /app
COPY requirements.txt .
RUN pip install --no-cache-dir -r requirements.txt
COPY csrc csrc
COPY vgate vgate
# compile every HIP kernel for gfx950 and link the in-tree extension (vgate/_C*.so)
RUN python csrc/build.py
COPY main.py config.yaml bench.py ./
COPY benchmarks benchmarks
EXPOSE 8000
HEALTHCHECK --interval=15s --timeout=5s --start-period=300s --retries=3 \
    CMD python -c "import urllib.request,sys; sys.exit(0 if urllib.request.urlopen('http://127.0.0.1:8000/health',timeout=4).status==200 else 1)"
CMD ["python", "main.py"]

FROM python:3.10-slim AS cpu
ENV PYTHONUNBUFFERED=1 \
    VGATE_DRY_RUN=true
WORKDIR /app
COPY requirements.txt .
RUN pip install --no-cache-dir -r requirements.txt && pip install --no-cache-dir torch --index-url https://download.pytorch.org/whl/cpu
COPY vgate vgate
COPY main.py config.yaml ./
EXPOSE 8000
HEALTHCHECK --interval=15s --timeout=5s --start-period=20s --retries=3 \
    CMD python -c "import urllib.request,sys; sys.exit(0 if urllib.request.urlopen('http://127.0.0.1:8000/health',timeout=4).status==200 else 1)"
CMD ["python", "main.py"]
