# MI355X (gfx950) image: ROCm PyTorch base, HIP kernels compiled at build time.
FROM rocm/pytorch:latest
ENV PYTHONDONTWRITEBYTECODE=1 PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 PYTORCH_ROCM_ARCH=gfx950
WORKDIR /app
RUN pip install --no-cache-dir fastapi uvicorn pydantic httpx prometheus_client safetensors pybind11
COPY ai_agent_kubectl_amd ./ai_agent_kubectl_amd
COPY __graft_entry__.py bench.py ./
RUN python -c "import __graft_entry__ as g; g.build()"
# optional: kubectl for POST /execute (the reference image did not ship it, quirk Q10)
# RUN curl -fsSLo /usr/local/bin/kubectl https://dl.k8s.io/release/v1.31.0/bin/linux/amd64/kubectl && chmod +x /usr/local/bin/kubectl
EXPOSE 8000
CMD ["python", "-m", "ai_agent_kubectl_amd.serve"]
