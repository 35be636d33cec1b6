"""REST API behaviour specs (reference tests/bot_tests/test_api.py:14-144), run against SQLite when
Django + DRF + django-mptt are installed (they are not in the CI image: skipped there)."""
import os

import pytest

django = pytest.importorskip("django")
pytest.importorskip("rest_framework")
pytest.importorskip("mptt")

pytestmark = pytest.mark.django

os.environ.setdefault("DJANGO_SETTINGS_MODULE", "tests.django_settings")
django.setup()

from django.core.management import call_command  # noqa: E402
from rest_framework.authtoken.models import Token  # noqa: E402
from rest_framework.test import APIClient  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def db():
    call_command("migrate", run_syncdb=True, verbosity=0)


@pytest.fixture
def client():
    from django.contrib.auth.models import User

    user, _ = User.objects.get_or_create(username="api")
    token, _ = Token.objects.get_or_create(user=user)
    c = APIClient()
    c.credentials(HTTP_AUTHORIZATION=f"Token {token.key}")
    return c


@pytest.fixture
def bot():
    from assistant.bot.models import Bot
    return Bot.objects.get_or_create(codename="default")[0]


def test_dialog_crud(client, bot):
    r = client.post("/api/v1/dialogs/", {"bot": "default"}, format="json")
    assert r.status_code == 201
    did = r.json()["id"]
    assert client.get(f"/api/v1/dialogs/{did}/").json()["bot"] == "default"
    assert client.patch(f"/api/v1/dialogs/{did}/", {"is_completed": True}, format="json").json()["is_completed"]
    assert client.delete(f"/api/v1/dialogs/{did}/").status_code == 204


def test_message_create_answers(client, bot):
    from assistant.ai.providers.fake import FakeAIProvider

    did = client.post("/api/v1/dialogs/", {"bot": "default"}, format="json").json()["id"]
    FakeAIProvider.reset()
    FakeAIProvider.script(["Test AI response"])
    r = client.post(f"/api/v1/dialogs/{did}/messages/", {"text": "hello"}, format="json")
    assert r.status_code == 201
    assert r.json()["text"] == "hello" and r.json()["answer"][0]["text"] == "Test AI response"
    assert len(client.get(f"/api/v1/dialogs/{did}/messages/").json()) == 2
