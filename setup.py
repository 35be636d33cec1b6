"""Package definition (mirrors /root/reference/setup.py:3-48, widened to the MI355X engine).

Installs the Django apps (``assistant.*``), the native engine (``django_assistant_bot_amd``, whose
gfx950 extension is compiled in-tree on first import or by ``python -m django_assistant_bot_amd.build``
-- the HIP / C++ sources ship as package data) and the model server (``gpu_service``).

    pip install --no-deps --no-build-isolation -e .      # editable (example/requirements.txt: -e ..)
    pip wheel --no-deps --no-build-isolation . -w dist    # wheel

The Python dependencies are optional per deployment (Django / DRF / Celery for the bot host,
FastAPI / uvicorn for gpu_service, torch-ROCm for the engine), so ``install_requires`` lists only
what every import path needs; ``extras_require`` names the rest.
"""
from setuptools import find_packages, setup

TEMPLATES = "templates/admin/broadcasting/broadcastcampaign"

setup(
    name="django-assistant-bot-amd",
    version="0.3.0",
    description="Django assistant-bot framework with an MI355X-native (gfx950 HIP) RAG engine",
    packages=find_packages(include=["assistant", "assistant.*", "django_assistant_bot_amd",
                                    "django_assistant_bot_amd.*", "gpu_service", "gpu_service.*"]),
    package_data={
        "assistant.bot": ["schemas/*.json"],
        "assistant.processing": ["schemas/*.json"],
        "assistant.broadcasting": ["workflow.md", f"{TEMPLATES}/*.html", f"{TEMPLATES}/includes/*.html"],
        "django_assistant_bot_amd": ["csrc/*.cpp", "csrc/kernels/*.hip", "csrc/kernels/*.h",
                                     "csrc/runtime/*.cpp", "csrc/runtime/*.h", "csrc/tests/*.cpp"],
        "gpu_service": ["requirements.txt", "bin/*.py"],
    },
    include_package_data=True,
    python_requires=">=3.10",
    install_requires=["numpy"],
    extras_require={
        "django": ["Django>=4.2", "djangorestframework>=3.15", "django-mptt>=0.16", "django-environ>=0.11",
                   "asgiref>=3.7"],
        "celery": ["celery[redis]>=5.3"],
        "postgres": ["psycopg[binary]>=3.1", "pgvector>=0.2"],
        "engine": ["torch", "tokenizers", "safetensors", "pybind11"],
        "service": ["fastapi", "uvicorn", "pydantic", "aiohttp", "prometheus_client"],
    },
    zip_safe=False,
)
