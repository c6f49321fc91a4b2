/*
 * fi_param_stub.h — the two parameter calls of libfabric's core
 * (fi_param_define / fi_param_get, src/var.c:188-231 and :290-360) for the
 * test owners, which load a provider without libfabric.so.  Same contract:
 * a parameter <name> of provider <prov> is the environment variable
 * FI_<PROV>_<NAME> in upper case; fi_param_get returns -FI_ENODATA when it
 * is unset and converts by the defined type (string: the variable's value,
 * int, bool: 0/1 from 0/1/yes/no/true/false/on/off, size_t).  Built with
 * -rdynamic so the provider's references resolve here.  Test code.
 */
#ifndef FI_PARAM_STUB_H
#define FI_PARAM_STUB_H
#include <ctype.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include <rdma/fabric.h>
#include <rdma/fi_errno.h>
#include <rdma/providers/fi_prov.h>

#define STUB_MAX_PARAMS 128
static struct stub_param {
	char env[128];
	char name[64];
	enum fi_param_type type;
	char help[320];
} stub_params[STUB_MAX_PARAMS];
static int stub_nparams;

static void stub_env_name(const struct fi_provider *prov, const char *name, char *out, size_t n)
{
	snprintf(out, n, "FI_%s_%s", prov ? prov->name : "", name);
	for (char *c = out; *c; c++)
		*c = (char)toupper((unsigned char)*c);
}

__attribute__((visibility("default"))) int fi_param_define(const struct fi_provider *provider,
							   const char *param_name,
							   enum fi_param_type type,
							   const char *help_string_fmt, ...)
{
	struct stub_param *p;
	va_list ap;

	if (!param_name || !help_string_fmt || !*help_string_fmt)
		return -FI_EINVAL;
	if (stub_nparams == STUB_MAX_PARAMS)
		return -FI_ENOMEM;
	p = &stub_params[stub_nparams++];
	stub_env_name(provider, param_name, p->env, sizeof(p->env));
	snprintf(p->name, sizeof(p->name), "%s", param_name);
	p->type = type;
	va_start(ap, help_string_fmt);
	vsnprintf(p->help, sizeof(p->help), help_string_fmt, ap);
	va_end(ap);
	return FI_SUCCESS;
}

__attribute__((visibility("default"))) int fi_param_get(struct fi_provider *provider,
							const char *param_name, void *value)
{
	char env[128];
	const struct stub_param *p = NULL;
	const char *v;

	stub_env_name(provider, param_name, env, sizeof(env));
	for (int i = 0; i < stub_nparams && !p; i++)
		if (!strcmp(stub_params[i].env, env))
			p = &stub_params[i];
	if (!p)
		return -FI_ENOENT;      /* not defined (var.c: "variable not found") */
	v = getenv(env);
	if (!v)
		return -FI_ENODATA;
	switch (p->type) {
	case FI_PARAM_STRING:
		*(const char **)value = v;
		return FI_SUCCESS;
	case FI_PARAM_INT:
		*(int *)value = atoi(v);
		return FI_SUCCESS;
	case FI_PARAM_SIZE_T:
		*(size_t *)value = (size_t)strtoull(v, NULL, 0);
		return FI_SUCCESS;
	case FI_PARAM_BOOL:
		if (!strcmp(v, "1") || !strcasecmp(v, "yes") || !strcasecmp(v, "true") ||
		    !strcasecmp(v, "on"))
			*(int *)value = 1;
		else if (!strcmp(v, "0") || !strcasecmp(v, "no") || !strcasecmp(v, "false") ||
			 !strcasecmp(v, "off"))
			*(int *)value = 0;
		else
			return -FI_EINVAL;
		return FI_SUCCESS;
	default:
		return -FI_EINVAL;
	}
}

/* `fi_info -e` for the defined parameters: one line each. */
static void stub_print_params(FILE *f)
{
	static const char *tn[] = { "String", "Integer", "Boolean (0/1, on/off, true/false, yes/no)",
				    "size_t" };

	for (int i = 0; i < stub_nparams; i++)
		fprintf(f, "PARAM %s %s: %s\n", stub_params[i].env,
			(unsigned)stub_params[i].type < 4 ? tn[stub_params[i].type] : "?",
			stub_params[i].help);
}
#endif
