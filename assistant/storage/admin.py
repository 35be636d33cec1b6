"""Knowledge-base admin classes (reference storage/admin.py:14-72); the host project registers them."""
from django.contrib import admin
from django.urls import reverse
from django.utils.html import format_html

from assistant.admin.admin import SuperUserMixin
from assistant.storage.models import Document, Question, Sentence, WikiDocument


class DocumentAdmin(SuperUserMixin, admin.ModelAdmin):
    list_display = ("id", "name", "section_display", "description")
    ordering = ("id",)
    readonly_fields = ("sentences_display", "questions_display")

    @admin.display(description="Section")
    def section_display(self, obj):
        if not obj.wiki_id:
            return "-"
        url = reverse("admin:assistant_storage_wikidocument_change", args=[obj.wiki_id])
        return format_html('<a href="{}">{}</a>', url, obj.wiki)

    @admin.display(description="Sentences")
    def sentences_display(self, obj):
        return format_html("<pre>{}</pre>", "\n".join(s.text for s in obj.sentences.order_by("id")))

    @admin.display(description="Questions")
    def questions_display(self, obj):
        return format_html("<pre>{}</pre>", "\n".join(q.text for q in obj.questions.order_by("id")))


class WikiDocumentAdmin(SuperUserMixin, admin.ModelAdmin):
    list_display = ("id", "path", "documents_link", "processing_status", "created_at")
    ordering = ("id",)
    list_filter = ("bot__codename", "processing__status")
    actions = ("process",)

    @admin.display(description="Documents")
    def documents_link(self, obj):
        return format_html('<a href="{}?wiki__id__exact={}">Documents ({})</a>',
                           reverse("admin:assistant_storage_document_changelist"), obj.id, obj.documents.count())

    @admin.display(description="Processing")
    def processing_status(self, obj):
        p = obj.processing.order_by("-id").first()
        return p.status if p else "-"

    @admin.action(description="Process")
    def process(self, request, queryset):
        for wiki in queryset:
            wiki.save(update_fields=["updated_at"])  # re-fires the ingest signal


class SentenceAdmin(admin.ModelAdmin):
    list_display = ("id", "text", "order")


class QuestionAdmin(admin.ModelAdmin):
    list_display = ("id", "text", "order")
